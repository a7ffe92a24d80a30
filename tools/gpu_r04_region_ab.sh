# k_sha per-lane region balance (BSG_REGION_LAG / BSG_REGION_POLL) with the early
# chains on: configs[1] + nested configs[2] bench lines per variant, two interleaved rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2; do
  for v in base lag1 lag6 poll4 poll16; do
    echo "== $v round $r" >> gpurun_out/r04_region_ab.log
    BSG_LIB_PATH=bs_amd/variants/lib_$v.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-sample-mib 0 --e2e-mib 0 >> gpurun_out/r04_region_ab.log 2>&1 || exit $?
  done
done
