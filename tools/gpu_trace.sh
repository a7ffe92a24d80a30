# rocprofv3 kernel trace + stats of the default bench (no pytest); PMC passes when PMC=1.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS=${BENCH_ARGS:-"--steps 5 --warmup 1 --cpu-sample-mib 0"}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof_trace.log 2>&1 || exit $?
if [ "${PMC:-0}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --cpu-sample-mib 0 > gpurun_out/prof_fetch.log 2>&1 && \
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --cpu-sample-mib 0 > gpurun_out/prof_write.log 2>&1
fi
