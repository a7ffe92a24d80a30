# A/B on one box: the asm k_scan loop (libbsgpu.so) against the compiled one (libbsgpu_noasm.so,
# -DBSG_SCAN_ASM2=0), configs[2] and configs[1], twice each, interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
A="--cpu-sample-mib 0 --e2e-mib 0"
for r in 1 2; do
  timeout -k 10 120 python bench.py --streams 256 --stream-mib 64 $A --steps 5 > gpurun_out/ab_asm_c2_$r.log 2>&1 || exit $?
  BSG_LIB_PATH=$GRAFT_REPO_ROOT/bs_amd/libbsgpu_noasm.so timeout -k 10 120 python bench.py --streams 256 --stream-mib 64 $A --steps 5 > gpurun_out/ab_cc_c2_$r.log 2>&1 || exit $?
  timeout -k 10 120 python bench.py $A > gpurun_out/ab_asm_c1_$r.log 2>&1 || exit $?
  BSG_LIB_PATH=$GRAFT_REPO_ROOT/bs_amd/libbsgpu_noasm.so timeout -k 10 120 python bench.py $A > gpurun_out/ab_cc_c1_$r.log 2>&1 || exit $?
done
