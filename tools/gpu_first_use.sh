# One-time HIP costs (tools/ubench/first_use) and the first-use costs of the drop-in Writer,
# each first-use case in fresh processes (box-to-box variance is large).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 60 ./tools/ubench/first_use > gpurun_out/first_use.log 2>&1 || exit $?
timeout -k 10 600 python tools/first_writer.py ${FW_CASES:-breakdown_init breakdown_init cold1m cold1m} > gpurun_out/first_writer.log 2>&1 || exit $?
