# Round 6, tenth GPU call: host copies in 1 MiB slices taken dynamically by the copy pool (a late
# or slow thread takes fewer) plus DMA stages on the GPU's NUMA node, against the previous head
# (one slice per thread, first-touch stages). call 9 showed the host copy rate bimodal between
# processes with the same placement (54-59 against 98-155 GB/s). e2e + Writer legs, four
# alternations, unpinned; then the host-copy and Writer tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
LEGS="--steps 5 --warmup 2 --configs2-steps 0 --cpu-sample-mib 0"
for i in 1 2 3 4; do
  BSG_LIB_PATH=bs_amd/ab/libbsgpu_head.so timeout -k 10 200 python -u bench.py $LEGS > gpurun_out/r06_c10_head_$i.log 2>&1 || exit $?
  timeout -k 10 200 python -u bench.py $LEGS > gpurun_out/r06_c10_new_$i.log 2>&1 || exit $?
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_host_copy.py tests/test_gpu_split_writer.py tests/test_gpu_concurrency.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_c10_pytest.log 2>&1 || exit $?
