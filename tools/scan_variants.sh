# Time experiment builds of libbsgpu (bs_amd/libbsgpu_v_*.so) with bench.py; then a kernel trace
# of the default build.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/variants.log
: > $out
for lib in bs_amd/libbsgpu.so bs_amd/libbsgpu_v_*.so; do
  for cfg in "" "--stream-mib 64 --streams 256"; do
    echo "== $lib $cfg" >> $out
    BSG_LIB_PATH=$PWD/$lib timeout -k 10 120 python bench.py --steps 5 --warmup 1 --cpu-sample-mib 0 $cfg >> $out 2>&1 || exit $?
  done
done
[ "${TRACE:-0}" = 1 ] && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --cpu-sample-mib 0 > gpurun_out/prof_trace.log 2>&1
