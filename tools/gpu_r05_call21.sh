# Round 5, twenty-first GPU call: young per-lane waves (BSG_LANE_YOUNG: 8 waves per k_sha
# workgroup, waves 4-7 per-lane only from each region's short end; the default library) against
# four waves (lib_noyoung): the whole GPU suite, then configs[2] and configs[1] A/B, three
# interleaved rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_pytest_gpu_call21.log 2>&1 || exit $?
for r in 1 2 3; do
  for v in new noyoung; do
    if [ $v = new ]; then lib=bs_amd/libbsgpu.so; else lib=bs_amd/variants/lib_$v.so; fi
    echo "== $v round $r" >> gpurun_out/r05_ab21_c2.log
    BSG_LIB_PATH=$lib timeout -k 10 120 python bench.py --streams 256 --stream-mib 64 --steps 10 --warmup 3 --cpu-sample-mib 0 --e2e-mib 0 >> gpurun_out/r05_ab21_c2.log 2>&1 || exit $?
    echo "== $v round $r" >> gpurun_out/r05_ab21_c1.log
    BSG_LIB_PATH=$lib timeout -k 10 120 python bench.py --steps 20 --warmup 5 --configs2-steps 0 --cpu-sample-mib 0 --e2e-mib 0 >> gpurun_out/r05_ab21_c1.log 2>&1 || exit $?
  done
done
