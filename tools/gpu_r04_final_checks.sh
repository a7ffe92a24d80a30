# Round 4 final checks at the final head: host TSan in GPU mode (Writers, Readers, a raw context
# and three engines with early chains at once), then 1,200 randomized parity draws (every 10th a
# 256-320 MiB engine run with the early chains).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 bash tools/tsan_host.sh gpu > gpurun_out/r04_tsan_gpu_final.log 2>&1 || exit $?
for b in 160000 161000; do
  timeout -k 10 500 python -u tools/stress_parity.py 600 $b >> gpurun_out/r04_stress_parity_final2.log 2>&1 || exit $?
done
