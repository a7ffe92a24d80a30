# k_scan / k_sha HBM traffic after the k_scan split (round 2): counter list, kernel-trace stats
# + FETCH_SIZE / WRITE_SIZE for configs[1] and configs[2], and the scan_calib calibration.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -s KILL 60 rocprofv3 -L > $O/rocprof_counters.txt 2>&1 || true
OUT=prof_c1 BENCH_ARGS="--cpu-sample-mib 0 --e2e-mib 0" bash tools/gpu_trace_args.sh || exit $?
OUT=prof_c2 bash tools/gpu_trace_args.sh || exit $?
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $O/calib_fetch -o run --output-format csv -- ./tools/ubench/scan_calib > $O/calib_fetch.log 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d $O/calib_write -o run --output-format csv -- ./tools/ubench/scan_calib > $O/calib_write.log 2>&1
