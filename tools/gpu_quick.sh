# Quick loop: GPU tests, both bench workloads, kernel-trace stats of both.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --cpu-sample-mib 0 --e2e-mib 0 > $O/bench_c1.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --streams 256 --stream-mib 64 --cpu-sample-mib 0 --e2e-mib 0 > $O/bench_c2.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/q_c1 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-sample-mib 0 --e2e-mib 0 > $O/q_c1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/q_c2 -o run --output-format csv -- python3 bench.py --streams 256 --stream-mib 64 --steps 3 --warmup 1 --cpu-sample-mib 0 --e2e-mib 0 > $O/q_c2.log 2>&1
