# Quick loop + FETCH_SIZE passes: GPU tests, both bench workloads, kernel-trace stats and
# FETCH_SIZE of both (separate passes).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
bash tools/gpu_quick.sh || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/qf_c1 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --cpu-sample-mib 0 --e2e-mib 0 > $O/qf_c1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/qf_c2 -o run --output-format csv -- python3 bench.py --streams 256 --stream-mib 64 --steps 1 --warmup 0 --cpu-sample-mib 0 --e2e-mib 0 > $O/qf_c2.log 2>&1
