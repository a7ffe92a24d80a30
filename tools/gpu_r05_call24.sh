# Round 5, twenty-fourth GPU call: e2e reps after the stage pool hands every stream the same
# buffers (bsg_reset returns the stages last first): two default bench lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/r05_bench_pool1.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r05_bench_pool2.log 2>&1
