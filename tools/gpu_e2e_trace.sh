# Kernel + memory-copy trace of the 1 GiB e2e streaming path (no counters), for
# tools/e2e_rep_timeline.py: python tools/e2e_rep_timeline.py gpurun_out/<OUT> 3
# OUT (e2e_trace) names the output directory; BSG_LIB_PATH (+ BSG_LIB_PARTIAL=1) traces a variant.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=${OUT:-e2e_trace}
TRACE="--kernel-trace --memory-copy-trace"
[ "${HIP_TRACE:-0}" = 1 ] && TRACE="$TRACE --hip-trace"
timeout -k 10 240 rocprofv3 $TRACE --output-format csv -d gpurun_out/$OUT -o run -- python3 tools/e2e_trace_run.py > gpurun_out/$OUT.log 2>&1 || exit $?
