# Round 6, eleventh GPU call: randomized parity at the round-6 head (the k_scan asm statement,
# the solo octet loop, the copy slicing): 600 seeded draws of batch, streaming and Writer runs
# against the oracle, every 10th a 256-320 MiB engine run with the early chains.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u tools/stress_parity.py 600 96000 > gpurun_out/r06_stress_parity.log 2>&1 || exit $?
