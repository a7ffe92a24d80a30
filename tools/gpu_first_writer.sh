# First-use costs of the drop-in Writer (tools/first_writer.py) and the pinned-staging
# microbenchmark (tools/ubench/pin_cost), on the MI355X.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 ./tools/ubench/pin_cost > gpurun_out/pin_cost.log 2>&1 || exit $?
timeout -k 10 600 python tools/first_writer.py ${FW_CASES:-} > gpurun_out/first_writer.log 2>&1 || exit $?
