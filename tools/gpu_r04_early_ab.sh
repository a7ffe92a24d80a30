# Early chains (KNOB_EARLY / BSG_EARLY): the -m gpu suite with them on (default), then an
# interleaved bench A/B on one box (BSG_EARLY=1 vs 0), three rounds, configs[1] + nested
# configs[2] without CPU baseline / e2e, a kernel trace of configs[2] (both streams), then
# randomized parity draws.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof_early
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04_pytest_gpu_early.log 2>&1 || exit $?
for r in 1 2 3; do
  for v in 1 0; do
    echo "== BSG_EARLY=$v round $r" >> gpurun_out/r04_early_ab.log
    BSG_EARLY=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-sample-mib 0 --e2e-mib 0 >> gpurun_out/r04_early_ab.log 2>&1 || exit $?
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_early/trace -o run --output-format csv -- python3 bench.py --streams 256 --stream-mib 64 --cpu-sample-mib 0 --e2e-mib 0 --steps 3 --warmup 1 > gpurun_out/prof_early/trace.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/stress_parity.py 300 131000 > gpurun_out/r04_stress_parity_early.log 2>&1
