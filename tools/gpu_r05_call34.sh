# Round 5, thirty-fourth GPU call: the step gap after BSG_KNOB_POLL (finish() polls its stream)
# and the GC off in the bench's step loop. A kernel + copy + HIP API trace of configs[1] (for
# tools/step_gaps.py), then configs[1] and configs[2] A/B against the blocking wait with the GC on
# (BSG_BENCH_POLL=0), three interleaved rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS="--steps 5 --warmup 2 --configs2-steps 0 --cpu-sample-mib 0 --e2e-mib 0"
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace -d gpurun_out/gaps34 -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/gaps34.log 2>&1 || exit $?
for r in 1 2 3; do
  for v in 1 0; do
    echo "== poll $v round $r" >> gpurun_out/r05_ab34_c1.log
    BSG_BENCH_POLL=$v timeout -k 10 120 python bench.py --steps 20 --warmup 5 --configs2-steps 0 --cpu-sample-mib 0 --e2e-mib 0 >> gpurun_out/r05_ab34_c1.log 2>&1 || exit $?
  done
done
for r in 1 2; do
  for v in 1 0; do
    echo "== poll $v round $r" >> gpurun_out/r05_ab34_c2.log
    BSG_BENCH_POLL=$v timeout -k 10 120 python bench.py --streams 256 --stream-mib 64 --steps 10 --warmup 3 --cpu-sample-mib 0 --e2e-mib 0 >> gpurun_out/r05_ab34_c2.log 2>&1 || exit $?
  done
done
