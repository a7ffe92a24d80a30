# Mid-round check: the GPU suite, the Writer A/B against the previous build, first-use costs,
# N concurrent Writers, and the host-TSan stress driver in GPU mode.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 900 python tools/writer_ab.py bs_amd/libbsgpu.so ${AB_VARIANTS:-} > gpurun_out/writer_ab.log 2>&1 || exit $?
timeout -k 10 600 python tools/first_writer.py cold1m cold1m first4g first4g first4g > gpurun_out/first_writer.log 2>&1 || exit $?
timeout -k 10 600 python tools/concurrent_writers.py > gpurun_out/concurrent_writers.log 2>&1 || exit $?
timeout -k 10 900 bash tools/tsan_host.sh gpu > gpurun_out/tsan_gpu.log 2>&1 || exit $?
