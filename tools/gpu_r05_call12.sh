# Round 5, twelfth GPU call: kernel trace + FETCH_SIZE / WRITE_SIZE passes of configs[1] and
# configs[2] with the current library, and the strip-pattern FETCH calibration (scan_calib).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=prof_c1 BENCH_ARGS="--cpu-sample-mib 0 --e2e-mib 0 --configs2-steps 0" bash tools/gpu_trace_args.sh || exit $?
OUT=prof_c2 bash tools/gpu_trace_args.sh || exit $?
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/calib -o run --output-format csv -- tools/ubench/scan_calib > gpurun_out/calib.log 2>&1
