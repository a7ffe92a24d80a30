# Round 5, fourth GPU call: the k_scan A/B of call 3 again (bench.py's traffic lookup had tripped
# over the new SQ summary), the streaming path's copy threads, the chain's second counter pass
# (wait / active / fetch level, on k_early and the bare octet loop), and a kernel trace of one
# configs[1] run with the round-5 schedule.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
python -m bs_amd.build
for r in 1 2 3; do
  for v in r4 new nosc noscwg load3 p3; do
    echo "== $v round $r" >> gpurun_out/r05_ab4.log
    if [ $v = new ]; then lib=bs_amd/libbsgpu.so; else lib=bs_amd/variants/lib_$v.so; fi
    BSG_LIB_PATH=$lib timeout -k 10 120 python bench.py --streams 256 --stream-mib 64 --steps 10 --warmup 3 --cpu-sample-mib 0 --e2e-mib 0 >> gpurun_out/r05_ab4.log 2>&1 || exit $?
  done
done
for r in 1 2 3; do
  for t in 8 12 16; do
    echo "== copy threads $t round $r" >> gpurun_out/r05_e2e_threads.log
    BSG_COPY_THREADS=$t E2E_REPS=6 timeout -k 10 120 python tools/e2e_trace_run.py >> gpurun_out/r05_e2e_threads.log 2>&1 || exit $?
  done
done
CTRS="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS SQ_IFETCH_LEVEL GRBM_GUI_ACTIVE"
timeout -s KILL 60 rocprofv3 --pmc $CTRS -d gpurun_out/pmc2_oct -o run --output-format csv -- tools/ubench/oct_pmc > gpurun_out/pmc2_oct.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc $CTRS -d gpurun_out/pmc2_c1 -o run --output-format csv -- python3 bench.py --cpu-sample-mib 0 --e2e-mib 0 --configs2-steps 0 --steps 1 --warmup 1 > gpurun_out/pmc2_c1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c1_r05 -o run --output-format csv -- python3 bench.py --cpu-sample-mib 0 --e2e-mib 0 --configs2-steps 0 --steps 3 --warmup 1 > gpurun_out/prof_c1_r05.log 2>&1
