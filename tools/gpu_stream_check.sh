# Streaming-path check after a change to bsg_ctx (staging ring, lazy engines): the streaming /
# Writer / window parity tests, first-use costs, the e2e rate and the default bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 900 $PYT tests -m gpu > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 600 python tools/first_writer.py > gpurun_out/first_writer.log 2>&1 || exit $?
timeout -k 10 300 python tools/e2e_bench.py > gpurun_out/e2e.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_default.log 2>&1 || exit $?
