# Round 6, sixth GPU call: small hasher batches with a long blob on the engine's chains (the
# Writer's tree nodes), bench.py with bsg_init up front; the tests that cover both, then two
# default bench lines (the driver's form).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_blob_hash.py tests/test_gpu_split_writer.py tests/test_gpu_bench_contract.py tests/test_gpu_host_copy.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r06_c6_pytest.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r06_c6_bench1.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r06_c6_bench2.log 2>&1 || exit $?
