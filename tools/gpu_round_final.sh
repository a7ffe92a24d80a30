# End-of-round evidence: GPU tests, smoke, bench lines (configs[1] default, configs[2]), e2e,
# and rocprofv3 kernel-trace + FETCH_SIZE/WRITE_SIZE passes for both workloads.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-sample-mib 1024 --e2e-mib 0 --stream-mib 64 --streams 256 > gpurun_out/bench_c2.log 2>&1 || exit $?
OUT=prof_c1 BENCH_ARGS="--cpu-sample-mib 0 --e2e-mib 0" bash tools/gpu_trace_args.sh || exit $?
OUT=prof_c2 bash tools/gpu_trace_args.sh || exit $?
timeout -k 10 300 python tools/e2e_bench.py > gpurun_out/e2e.log 2>&1
