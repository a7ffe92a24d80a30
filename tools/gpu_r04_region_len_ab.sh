# k_sha per-lane region poll by next-job length (BSG_REGION_BY_LEN, lag 3 / 10 / 25 %) against the
# share-taken poll (base), configs[2] lines, three interleaved rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in base len3 len10 len25; do
    echo "== $v round $r" >> gpurun_out/r04_region_len_ab.log
    BSG_LIB_PATH=bs_amd/variants/lib_$v.so timeout -k 10 200 python bench.py --streams 256 --stream-mib 64 --steps 20 --warmup 5 --cpu-sample-mib 0 --e2e-mib 0 >> gpurun_out/r04_region_len_ab.log 2>&1 || exit $?
  done
done
