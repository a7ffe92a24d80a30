# k_start (one set-up dispatch per run): the -m gpu suite, the event-cost / step-time
# measurement, a configs[1] kernel trace, and two default bench lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/kstart
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04_pytest_gpu_kstart.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/profile_cost.py > gpurun_out/r04_profile_cost_kstart.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kstart/c1 -o run --output-format csv -- python3 bench.py --cpu-sample-mib 0 --e2e-mib 0 --configs2-steps 0 --steps 3 --warmup 1 > gpurun_out/kstart/c1.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r04_bench_kstart1.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r04_bench_kstart2.log 2>&1
