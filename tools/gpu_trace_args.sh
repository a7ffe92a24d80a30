# rocprofv3 kernel trace + stats and the FETCH_SIZE / WRITE_SIZE passes for one bench workload.
# BENCH_ARGS selects the workload, OUT the gpurun_out subdirectory.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${OUT:-prof_c2}
mkdir -p $OUT
export TMPDIR=/tmp
ARGS=${BENCH_ARGS:-"--streams 256 --stream-mib 64 --cpu-sample-mib 0 --e2e-mib 0"}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_trace -o run --output-format csv -- python3 bench.py $ARGS --steps 3 --warmup 1 > $OUT/prof_trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/prof_fetch -o run --output-format csv -- python3 bench.py $ARGS --steps 1 --warmup 0 > $OUT/prof_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/prof_write -o run --output-format csv -- python3 bench.py $ARGS --steps 1 --warmup 0 > $OUT/prof_write.log 2>&1
