# Round 6, the last head: host ThreadSanitizer in GPU mode (the host code changed since call 12:
# copy slicing, stage placement, first_flush, the hasher's engine route) and 600 more randomized
# parity draws (new seeds).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TSAN_OUT=$GRAFT_REPO_ROOT/tsan_build timeout -k 10 900 bash tools/tsan_host.sh gpu > gpurun_out/r06_tsan_gpu_last.log 2>&1 || exit $?
timeout -k 10 900 python -u tools/stress_parity.py 600 98000 > gpurun_out/r06_stress_parity_last.log 2>&1 || exit $?
