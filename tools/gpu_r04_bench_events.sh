# bench.py with the timed steps carrying only the SHA-256 stage's two HIP events: the bench
# contract tests, the event-cost measurement and two default lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench_contract.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04_pytest_bench_contract.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/profile_cost.py > gpurun_out/r04_profile_cost.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r04_bench_events1.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r04_bench_events2.log 2>&1
