# Round 6, the last head: the whole GPU suite and smoke after the k_lens atomics change, and one
# default bench line (the driver's form).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06_pytest_gpu_last.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_smoke_last.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r06_bench_last.log 2>&1 || exit $?
