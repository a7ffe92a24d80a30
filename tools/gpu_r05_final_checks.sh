# Round 5 final checks at the final head: 1,200 randomized parity draws (every 10th a 256-320 MiB
# engine run with the early chains) over the round-5 kernels (k_scan by ticket, k_prefix1, the
# fused exact pass, the aligned chain loops, per-lane SHA-256 from the generated statement),
# then host TSan in GPU mode.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for b in 170000 171000; do
  timeout -k 10 500 python -u tools/stress_parity.py 600 $b >> gpurun_out/r05_stress_parity_final.log 2>&1 || exit $?
done
timeout -k 10 600 bash tools/tsan_host.sh gpu > gpurun_out/r05_tsan_gpu_final.log 2>&1
