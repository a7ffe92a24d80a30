# Round 6, fourteenth GPU call: the stream's first 8 MiB staged go to the device at once
# (first_flush) instead of when the first 64 MiB stage is full, against the previous head
# (bs_amd/ab/libbsgpu_head.so). e2e + Writer legs, four alternations; then the streaming,
# Writer and host-copy tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
LEGS="--steps 5 --warmup 2 --configs2-steps 0 --cpu-sample-mib 0"
for i in 1 2 3 4; do
  BSG_LIB_PATH=bs_amd/ab/libbsgpu_head.so timeout -k 10 200 python -u bench.py $LEGS > gpurun_out/r06_c14_head_$i.log 2>&1 || exit $?
  timeout -k 10 200 python -u bench.py $LEGS > gpurun_out/r06_c14_new_$i.log 2>&1 || exit $?
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_host_copy.py tests/test_gpu_split_writer.py tests/test_gpu_parity.py tests/test_gpu_params.py tests/test_gpu_large_streams.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_c14_pytest.log 2>&1 || exit $?
