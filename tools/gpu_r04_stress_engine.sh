# Randomized parity with the engine draws (every 10th: a 256-320 MiB device-resident run, early
# chains on), two processes of 200 draws.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for b in 140000 141000; do
  timeout -k 10 500 python -u tools/stress_parity.py 200 $b >> gpurun_out/r04_stress_parity_engine.log 2>&1 || exit $?
done
