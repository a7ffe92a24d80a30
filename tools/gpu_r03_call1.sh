# Round-3 GPU call 1: the GPU suite, host TSan in GPU mode, the Writer A/B, N concurrent
# Writers (default copy pool and 16 copy threads) and first-use costs.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 600 bash tools/tsan_host.sh gpu > gpurun_out/tsan_gpu.log 2>&1 || exit $?
timeout -k 10 600 python tools/writer_ab.py bs_amd/libbsgpu.so ${AB_VARIANTS:-} > gpurun_out/writer_ab.log 2>&1 || exit $?
timeout -k 10 300 python tools/concurrent_writers.py > gpurun_out/concurrent_writers.log 2>&1 || exit $?
BSG_COPY_THREADS=16 timeout -k 10 300 python tools/concurrent_writers.py > gpurun_out/concurrent_writers_16.log 2>&1 || exit $?
timeout -k 10 300 python tools/first_writer.py cold1m cold1m first4g first4g first4g > gpurun_out/first_writer.log 2>&1 || exit $?
