# Round 5, thirtieth GPU call: configs[2]'s group-ticket threshold (BSG_TLEN_PCT: jobs of at
# least this % of the longest run 8 per wave on octet chains, below it 32 per wave on pairs)
# 53, 56 and 58: the octet tier costs ~3x the per-lane wave-cycles per block and
# the pair tier about the same, so jobs that a pair still finishes before the longest chain are
# cheaper there. Three interleaved rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in tlen53 tlen56 tlen58; do
    if [ $v = new ]; then lib=bs_amd/libbsgpu.so; else lib=bs_amd/variants/lib_$v.so; fi
    echo "== $v round $r" >> gpurun_out/r05_ab30_c2.log
    BSG_LIB_PATH=$lib timeout -k 10 120 python bench.py --streams 256 --stream-mib 64 --steps 10 --warmup 3 --cpu-sample-mib 0 --e2e-mib 0 >> gpurun_out/r05_ab30_c2.log 2>&1 || exit $?
  done
done
