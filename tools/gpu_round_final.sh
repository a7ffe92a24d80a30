# End-of-round evidence: GPU tests, smoke, two default bench lines (configs[1] + nested configs[2]), e2e,
# and rocprofv3 kernel-trace + FETCH_SIZE/WRITE_SIZE passes for both workloads.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_default.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_default2.log 2>&1 || exit $?
# configs[1] alone (no nested configs[2] leg) and configs[2] alone, for the kernel trace and PMC
OUT=prof_c1 BENCH_ARGS="--cpu-sample-mib 0 --e2e-mib 0 --configs2-steps 0" bash tools/gpu_trace_args.sh || exit $?
OUT=prof_c2 bash tools/gpu_trace_args.sh || exit $?
timeout -k 10 300 python tools/e2e_bench.py > gpurun_out/e2e.log 2>&1
