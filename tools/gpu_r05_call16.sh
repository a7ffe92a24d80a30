# Round 5, sixteenth GPU call: per-lane blocks per iteration (BSG_LANE_BPI 2 = default, 3, 4),
# configs[2] and configs[1], two interleaved rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for v in new bpi3 bpi4; do
    if [ $v = new ]; then lib=bs_amd/libbsgpu.so; else lib=bs_amd/variants/lib_$v.so; fi
    echo "== $v round $r" >> gpurun_out/r05_ab16_c2.log
    BSG_LIB_PATH=$lib timeout -k 10 120 python bench.py --streams 256 --stream-mib 64 --steps 10 --warmup 3 --cpu-sample-mib 0 --e2e-mib 0 >> gpurun_out/r05_ab16_c2.log 2>&1 || exit $?
    echo "== $v round $r" >> gpurun_out/r05_ab16_c1.log
    BSG_LIB_PATH=$lib timeout -k 10 120 python bench.py --steps 20 --warmup 5 --configs2-steps 0 --cpu-sample-mib 0 --e2e-mib 0 >> gpurun_out/r05_ab16_c1.log 2>&1 || exit $?
  done
done
