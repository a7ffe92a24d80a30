# Round 6, fifteenth GPU call: the Writer's Close hashes the tree nodes finished before the last
# tiles on a second hasher while those tiles run (Writer::PreHash), against the previous head
# (bs_amd/ab/libbsgpu_head.so). Writer + e2e legs, four alternations; the Writer tests; host
# ThreadSanitizer in GPU mode (the pre-hash is a host thread beside the background Put thread).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
LEGS="--steps 5 --warmup 2 --configs2-steps 0 --cpu-sample-mib 0"
for i in 1 2 3 4; do
  BSG_LIB_PATH=bs_amd/ab/libbsgpu_head.so timeout -k 10 200 python -u bench.py $LEGS > gpurun_out/r06_c15_head_$i.log 2>&1 || exit $?
  timeout -k 10 200 python -u bench.py $LEGS > gpurun_out/r06_c15_new_$i.log 2>&1 || exit $?
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_split_writer.py tests/test_gpu_host_copy.py tests/test_gpu_concurrency.py tests/test_gpu_filestore.py tests/test_gpu_large_streams.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_c15_pytest.log 2>&1 || exit $?
TSAN_OUT=$GRAFT_REPO_ROOT/tsan_build timeout -k 10 900 bash tools/tsan_host.sh gpu > gpurun_out/r06_c15_tsan_gpu.log 2>&1 || exit $?
