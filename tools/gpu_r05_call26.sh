# Round 5, twenty-sixth GPU call: per-lane block loads with one address and selector per iteration
# (BSG_LANE_LOADN, the default library) against lib_noloadn: the GPU suite, the instruction mix with
# every job per-lane, then configs[2] and configs[1] A/B, three interleaved rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_pytest_gpu_call26.log 2>&1 || exit $?
ARGS="--streams 256 --stream-mib 64 --cpu-sample-mib 0 --e2e-mib 0 --steps 1 --warmup 0"
BSG_LONG_MODE=off timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_INSTS_VMEM -d gpurun_out/lanemix26 -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/lanemix26.log 2>&1 || exit $?
for r in 1 2 3; do
  for v in new noloadn; do
    if [ $v = new ]; then lib=bs_amd/libbsgpu.so; else lib=bs_amd/variants/lib_$v.so; fi
    echo "== $v round $r" >> gpurun_out/r05_ab26_c2.log
    BSG_LIB_PATH=$lib timeout -k 10 120 python bench.py --streams 256 --stream-mib 64 --steps 10 --warmup 3 --cpu-sample-mib 0 --e2e-mib 0 >> gpurun_out/r05_ab26_c2.log 2>&1 || exit $?
  done
done
for r in 1 2; do
  for v in new noloadn; do
    if [ $v = new ]; then lib=bs_amd/libbsgpu.so; else lib=bs_amd/variants/lib_$v.so; fi
    echo "== $v round $r" >> gpurun_out/r05_ab26_c1.log
    BSG_LIB_PATH=$lib timeout -k 10 120 python bench.py --steps 20 --warmup 5 --configs2-steps 0 --cpu-sample-mib 0 --e2e-mib 0 >> gpurun_out/r05_ab26_c1.log 2>&1 || exit $?
  done
done
