# Round 5, thirty-eighth GPU call: k_scan with one 512-thread workgroup per CU (lib_wgs512,
# BSG_SCAN_WGS=512) against two 256-thread ones (the default) on configs[1], where the two
# workgroups of a CU end up to 2x apart (profiles/r05_scan_stamps36_wg.log); three rounds each.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in def wgs512; do
    if [ $v = def ]; then lib=bs_amd/libbsgpu.so; else lib=bs_amd/variants/lib_$v.so; fi
    echo "== $v round $r" >> gpurun_out/r05_ab38_c1.log
    BSG_LIB_PATH=$lib timeout -k 10 120 python bench.py --steps 20 --warmup 5 --configs2-steps 0 --cpu-sample-mib 0 --e2e-mib 0 >> gpurun_out/r05_ab38_c1.log 2>&1 || exit $?
  done
done
