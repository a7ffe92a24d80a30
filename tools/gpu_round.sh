# GPU check used between optimisation steps: parity tests, bench (configs[1] and [2]), e2e.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
[ "${SKIP_TESTS:-0}" = 1 ] || timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-sample-mib 0 > gpurun_out/bench_c1.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-sample-mib 0 --stream-mib 64 --streams 256 > gpurun_out/bench_c2.log 2>&1 && \
timeout -k 10 300 python tools/e2e_bench.py > gpurun_out/e2e.log 2>&1
rc=$?
echo "exit=$rc" >> gpurun_out/pytest_gpu.log
exit $rc
