# Round 5, twenty-eighth GPU call: 1,200 randomized parity draws at the head (after the per-lane
# loop's ballot guards and shared load base), new seeds.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for b in 180000 181000; do
  timeout -k 10 500 python -u tools/stress_parity.py 600 $b >> gpurun_out/r05_stress_parity_head.log 2>&1 || exit $?
done
