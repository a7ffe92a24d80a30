# Aggregate throughput of N concurrent split.Writers (tools/concurrent_writers.py) and the host
# TSan stress driver in GPU mode.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python tools/concurrent_writers.py > gpurun_out/concurrent_writers.log 2>&1 || exit $?
timeout -k 10 900 bash tools/tsan_host.sh gpu > gpurun_out/tsan_gpu.log 2>&1 || exit $?
