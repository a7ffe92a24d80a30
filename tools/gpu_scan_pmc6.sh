# Clock during k_scan (bench, configs[2]) and its replay: GRBM_COUNT / GRBM_GUI_ACTIVE per
# dispatch against the dispatch's duration.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
C="GRBM_COUNT GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/pmc6_bench -o run --output-format csv -- python3 bench.py --streams 256 --stream-mib 64 --steps 2 --warmup 1 --cpu-sample-mib 0 --e2e-mib 0 > gpurun_out/pmc6_bench.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/pmc6_replay -o run --output-format csv -- ./tools/ubench/scanload > gpurun_out/pmc6_replay.log 2>&1
