# Round-2 evidence: GPU tests, bench lines (configs[1], configs[2]), rocprofv3 kernel-trace
# stats and FETCH_SIZE / WRITE_SIZE passes for both workloads, and the FETCH_SIZE calibration
# of k_scan's load pattern (tools/ubench/scan_calib).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $O/bench_c1.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --streams 256 --stream-mib 64 --e2e-mib 0 > $O/bench_c2.log 2>&1 || exit $?
OUT=prof_c1 BENCH_ARGS="--cpu-sample-mib 0 --e2e-mib 0" bash tools/gpu_trace_args.sh || exit $?
OUT=prof_c2 bash tools/gpu_trace_args.sh || exit $?
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $O/calib_fetch -o run --output-format csv -- ./tools/ubench/scan_calib > $O/calib_fetch.log 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d $O/calib_write -o run --output-format csv -- ./tools/ubench/scan_calib > $O/calib_write.log 2>&1
timeout -k 10 300 python tools/writer_bench.py > $O/writer_bench.log 2>&1 || exit $?
E2E_TILES=256 timeout -k 10 300 python tools/e2e_bench.py > $O/e2e.log 2>&1
