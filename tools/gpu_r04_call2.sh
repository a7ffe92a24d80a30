# Round 4, after the boundary changes: the whole -m gpu suite, 600 randomized parity draws (a third
# of the streaming / Writer draws at stream offsets past 2^40), smoke, and the GPU-mode host TSan
# driver (Reader read-ahead and hasher changes).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04_pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/stress_parity.py 600 91000 > gpurun_out/r04_stress_parity.log 2>&1 || exit $?
timeout -k 10 400 bash tools/tsan_host.sh gpu > gpurun_out/r04_tsan_gpu.log 2>&1
