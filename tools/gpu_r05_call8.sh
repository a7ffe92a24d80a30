# Round 5, eighth GPU call: per-lane SHA-256 as one aligned asm statement (BSG_LANE_ASM=1,
# bs_amd/variants/lib_laneasm.so). The microbenchmark first (cycles per block, digests), then
# the GPU suite on the variant, then bench A/B against the default library, two rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 tools/ubench/lanes_align > gpurun_out/r05_lanes_align.log 2>&1 || exit $?
BSG_LIB_PATH=bs_amd/variants/lib_laneasm.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_pytest_gpu_laneasm.log 2>&1 || exit $?
for r in 1 2; do
  for v in new laneasm; do
    if [ $v = new ]; then lib=bs_amd/libbsgpu.so; else lib=bs_amd/variants/lib_$v.so; fi
    echo "== $v round $r" >> gpurun_out/r05_ab8.log
    BSG_LIB_PATH=$lib timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-sample-mib 0 --e2e-mib 0 >> gpurun_out/r05_ab8.log 2>&1 || exit $?
  done
done
