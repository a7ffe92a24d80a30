# Round 5, ninth GPU call: the per-lane asm variants (V1 aligned, V2 no st copies, V3 K through
# an SGPR = the product now) in the microbenchmark at one and two waves per SIMD, the GPU suite on
# the product (V3), then bench A/B of V3 (default library) against V1 (lib_laneasm), two rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 tools/ubench/lanes_align 1 > gpurun_out/r05_lanes_variants.log 2>&1 || exit $?
timeout -k 10 120 tools/ubench/lanes_align 2 >> gpurun_out/r05_lanes_variants.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_pytest_gpu_call9.log 2>&1 || exit $?
for r in 1 2; do
  for v in new laneasm; do
    if [ $v = new ]; then lib=bs_amd/libbsgpu.so; else lib=bs_amd/variants/lib_$v.so; fi
    echo "== $v round $r" >> gpurun_out/r05_ab9.log
    BSG_LIB_PATH=$lib timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-sample-mib 0 --e2e-mib 0 >> gpurun_out/r05_ab9.log 2>&1 || exit $?
  done
done
