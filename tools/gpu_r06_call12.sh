# Round 6, twelfth GPU call: host ThreadSanitizer in GPU mode at the round-6 head (8 split::Writers,
# a raw context and 8 verifying Readers at once over shared pools; the copy slicing, the hasher's
# engine route and the stage placement are host code). The instrumented library and driver were
# built in this container (TSAN_OUT=tsan_build, tools/tsan_host.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TSAN_OUT=$GRAFT_REPO_ROOT/tsan_build timeout -k 10 900 bash tools/tsan_host.sh gpu > gpurun_out/r06_tsan_gpu.log 2>&1 || exit $?
