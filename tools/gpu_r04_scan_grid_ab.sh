# A/B of k_scan's grid (BSG_SCAN_GRID workgroups per CU: 2 = default, 1, 4), same box,
# interleaved, two rounds; configs[1] + nested configs[2] bench lines without CPU baseline / e2e.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2; do
  for v in base scan1 scan4; do
    echo "== $v round $r" >> gpurun_out/r04_scan_grid_ab.log
    BSG_LIB_PATH=bs_amd/variants/lib_$v.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-sample-mib 0 --e2e-mib 0 >> gpurun_out/r04_scan_grid_ab.log 2>&1 || exit $?
  done
done
