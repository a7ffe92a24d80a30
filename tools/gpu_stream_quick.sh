# Quick streaming-path measurement: first-use costs and the e2e rates (no tests).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python tools/first_writer.py cold1m first4g > gpurun_out/first_writer.log 2>&1 || exit $?
timeout -k 10 300 python tools/e2e_bench.py > gpurun_out/e2e.log 2>&1 || exit $?
