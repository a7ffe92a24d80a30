set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_split_writer.py tests/test_gpu_filestore.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_cold.log 2>&1 || exit $?
timeout -k 10 200 python tools/cold_start.py > gpurun_out/cold.log 2>&1 || exit $?
timeout -k 10 300 python tools/e2e_bench.py > gpurun_out/e2e.log 2>&1
