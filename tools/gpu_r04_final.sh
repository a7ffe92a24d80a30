# Round 4 evidence at the final head, part A: the -m gpu suite, smoke, two default bench lines
# (configs[1] + nested configs[2], oracle_check on the bench's own bytes and on the e2e records),
# 600 more randomized parity draws.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04_pytest_gpu_final.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_smoke_final.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r04_bench_default.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r04_bench_default2.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/stress_parity.py 600 97000 > gpurun_out/r04_stress_parity_final.log 2>&1
