# Round 6 end-of-round evidence: the GPU suite, smoke, two default bench lines (the driver's forms),
# kernel traces + FETCH_SIZE / WRITE_SIZE passes and TCC_EA0_RDREQ-by-size passes for configs[1]
# and configs[2], and the SQ counters behind configs[2]'s work_roofline.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06_pytest_gpu_final.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_smoke_final.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r06_bench_final.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/r06_bench_default_args.log 2>&1 || exit $?
OUT=prof_c1 BENCH_ARGS="--cpu-sample-mib 0 --e2e-mib 0 --no-writer-e2e --configs2-steps 0" bash tools/gpu_trace_args.sh || exit $?
OUT=prof_c2 BENCH_ARGS="--streams 256 --stream-mib 64 --cpu-sample-mib 0 --e2e-mib 0 --no-writer-e2e" bash tools/gpu_trace_args.sh || exit $?
PMC="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
timeout -s KILL 200 rocprofv3 --pmc $PMC -d gpurun_out/rdreq_final_c1 -o run --output-format csv -- python3 bench.py --cpu-sample-mib 0 --e2e-mib 0 --no-writer-e2e --configs2-steps 0 --steps 1 --warmup 0 > gpurun_out/rdreq_final_c1.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc $PMC -d gpurun_out/rdreq_final_c2 -o run --output-format csv -- python3 bench.py --streams 256 --stream-mib 64 --cpu-sample-mib 0 --e2e-mib 0 --no-writer-e2e --steps 1 --warmup 0 > gpurun_out/rdreq_final_c2.log 2>&1 || exit $?
CTRS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_IFETCH GRBM_GUI_ACTIVE"
timeout -s KILL 180 rocprofv3 --pmc $CTRS -d gpurun_out/pmc_final_c2 -o run --output-format csv -- python3 bench.py --streams 256 --stream-mib 64 --cpu-sample-mib 0 --e2e-mib 0 --no-writer-e2e --steps 1 --warmup 1 > gpurun_out/pmc_final_c2.log 2>&1 || exit $?
