# Writer paths after a change: the Writer A/B against a variant, N concurrent Writers with the
# default copy pool and with 16 copy threads, then the host-TSan driver in GPU mode.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python tools/writer_ab.py bs_amd/libbsgpu.so ${AB_VARIANTS:-} > gpurun_out/writer_ab.log 2>&1 || exit $?
timeout -k 10 600 python tools/concurrent_writers.py > gpurun_out/concurrent_writers.log 2>&1 || exit $?
BSG_COPY_THREADS=16 timeout -k 10 600 python tools/concurrent_writers.py > gpurun_out/concurrent_writers_16.log 2>&1 || exit $?
timeout -k 10 900 bash tools/tsan_host.sh gpu > gpurun_out/tsan_gpu.log 2>&1 || exit $?
