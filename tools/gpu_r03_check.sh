# Round-3 check on the MI355X: the new concurrency / device-error / store tests first, then the
# whole GPU suite, smoke(), the driver's default bench line (configs[1] + nested configs[2]) and
# the host-TSan stress driver in GPU mode (8 Writers, a raw context, verifying Readers at once).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_gpu_device_error.py tests/test_gpu_concurrency.py \
  "tests/test_gpu_split_writer.py::test_memstore_does_not_keep_pieces_alive_for_few_chunks" \
  > gpurun_out/pytest_new.log 2>&1 || exit $?
timeout -k 10 900 $PYT tests -m gpu > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_default.log 2>&1 || exit $?
if [ "${TSAN:-1}" = 1 ]; then
  timeout -k 10 900 bash tools/tsan_host.sh gpu > gpurun_out/tsan_gpu.log 2>&1 || exit $?
fi
