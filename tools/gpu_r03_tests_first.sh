# The whole GPU suite, then the first-use costs (tools/first_writer.py) in fresh processes.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 600 python tools/first_writer.py breakdown_init breakdown_init cold1m cold1m cold1m first4g first4g first4g > gpurun_out/first_writer.log 2>&1 || exit $?
