# Round 5, thirty-first GPU call: is the e2e leg's slow mode (every rep ~32 ms instead of ~28.3)
# the state the configs[2] leg leaves behind? The bench without configs[2], then with, twice.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  echo "== no configs2, round $r" >> gpurun_out/r05_e2e_order.log
  timeout -k 10 300 python bench.py --configs2-steps 0 --cpu-sample-mib 0 >> gpurun_out/r05_e2e_order.log 2>&1 || exit $?
  echo "== with configs2, round $r" >> gpurun_out/r05_e2e_order.log
  timeout -k 10 400 python bench.py --cpu-sample-mib 0 >> gpurun_out/r05_e2e_order.log 2>&1 || exit $?
done
