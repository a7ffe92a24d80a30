# Round 6 end-of-round profiles (the trace / PMC half of tools/gpu_r06_final.sh) with
# BSG_BENCH_INIT=0: bsg_init's warm-up launches (small k_scan / k_sha runs) otherwise enter the
# per-launch averages of the kernel statistics and the counter passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
export BSG_BENCH_INIT=0
OUT=prof_c1 BENCH_ARGS="--cpu-sample-mib 0 --e2e-mib 0 --no-writer-e2e --configs2-steps 0" bash tools/gpu_trace_args.sh || exit $?
OUT=prof_c2 BENCH_ARGS="--streams 256 --stream-mib 64 --cpu-sample-mib 0 --e2e-mib 0 --no-writer-e2e" bash tools/gpu_trace_args.sh || exit $?
PMC="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
timeout -s KILL 200 rocprofv3 --pmc $PMC -d gpurun_out/rdreq_final_c1 -o run --output-format csv -- python3 bench.py --cpu-sample-mib 0 --e2e-mib 0 --no-writer-e2e --configs2-steps 0 --steps 1 --warmup 0 > gpurun_out/rdreq_final_c1.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc $PMC -d gpurun_out/rdreq_final_c2 -o run --output-format csv -- python3 bench.py --streams 256 --stream-mib 64 --cpu-sample-mib 0 --e2e-mib 0 --no-writer-e2e --steps 1 --warmup 0 > gpurun_out/rdreq_final_c2.log 2>&1 || exit $?
CTRS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_IFETCH GRBM_GUI_ACTIVE"
timeout -s KILL 180 rocprofv3 --pmc $CTRS -d gpurun_out/pmc_final_c2 -o run --output-format csv -- python3 bench.py --streams 256 --stream-mib 64 --cpu-sample-mib 0 --e2e-mib 0 --no-writer-e2e --steps 1 --warmup 1 > gpurun_out/pmc_final_c2.log 2>&1 || exit $?
