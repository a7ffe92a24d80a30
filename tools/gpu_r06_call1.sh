# Round 6, first GPU call: the host-copy tests (non-temporal Write copies, stream stats, Writer
# timings), the streaming / Writer parity tests beside them, an interleaved A/B of the copy forms
# on the e2e and Writer legs, and one default bench line (the driver's form).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_host_copy.py tests/test_gpu_ownership.py tests/test_gpu_split_writer.py tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r06_c1_pytest.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/host_copy_ab.py 3 > gpurun_out/r06_c1_copy_ab.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r06_c1_bench.log 2>&1 || exit $?
