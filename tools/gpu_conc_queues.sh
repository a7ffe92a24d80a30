# N concurrent Writers with the default 4 hardware queues per process and with 16
# (GPU_MAX_HW_QUEUES), plus the Writer/raw A/B against a variant.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python tools/concurrent_writers.py > gpurun_out/concurrent_writers.log 2>&1 || exit $?
GPU_MAX_HW_QUEUES=16 timeout -k 10 300 python tools/concurrent_writers.py > gpurun_out/concurrent_writers_q16.log 2>&1 || exit $?
timeout -k 10 600 python tools/writer_ab.py bs_amd/libbsgpu.so ${AB_VARIANTS:-} > gpurun_out/writer_ab.log 2>&1 || exit $?
