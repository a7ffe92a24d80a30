# Round 4: a long randomized parity run at the final head (2,000 draws; a third of the streaming
# and Writer draws at stream offsets past 2^40), in 4 processes run one after the other.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for b in 101000 101500 102000 102500; do
  timeout -k 10 280 python -u tools/stress_parity.py 500 $b >> gpurun_out/r04_stress_parity_long.log 2>&1 || exit $?
done
