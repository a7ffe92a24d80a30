# Round 5, twenty-third GPU call: the per-lane loop's top vmcnt(0) wait measured from inside
# (BSG_LANE_DIAG build, diag2[0] = wait cycles, diag2[1] = per-lane cycles, summed over waves) on
# configs[2] as is and with every job per-lane; then one default bench line (e2e reps without GC).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
BSG_DIAG_RAW=1 BSG_LIB_PATH=bs_amd/variants/lib_lanediag.so timeout -k 10 120 python bench.py --streams 256 --stream-mib 64 --steps 3 --warmup 1 --cpu-sample-mib 0 --e2e-mib 0 > gpurun_out/r05_lanewait.log 2>&1 || exit $?
BSG_LONG_MODE=off BSG_DIAG_RAW=1 BSG_LIB_PATH=bs_amd/variants/lib_lanediag.so timeout -k 10 120 python bench.py --streams 256 --stream-mib 64 --steps 3 --warmup 1 --cpu-sample-mib 0 --e2e-mib 0 >> gpurun_out/r05_lanewait.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/r05_bench_gc.log 2>&1
