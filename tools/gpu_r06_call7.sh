# Round 6, seventh GPU call: small hasher batches with a long blob on the engine with every blob
# on a wave ticket (long mode 2 for the batch); latency per call for the Writer's node shape, the
# tests covering it, one bench line (writer_e2e's node_hash_ms).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_blob_hash.py tests/test_gpu_split_writer.py "tests/test_gpu_parity.py::test_sha_path_forced" -x -v --timeout 300 --timeout-method thread > gpurun_out/r06_c7_pytest.log 2>&1 || exit $?
for L in 15000 30000 50000 120000; do
  HS_N=63 HS_SIZE=11000 HS_LONG=$L timeout -k 10 120 python -u tools/hasher_small_bench.py >> gpurun_out/r06_c7_hasher.log 2>&1 || exit $?
done
HS_N=63 HS_SIZE=11000 HS_LONG=50000 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r06_c7_trace -o run --output-format csv -- python3 tools/hasher_small_bench.py > gpurun_out/r06_c7_trace.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r06_c7_bench.log 2>&1 || exit $?
