# Round 6, ninth GPU call: DMA staging placed on the GPU's NUMA node (PinBuf::alloc mbind,
# MPOL_PREFERRED) against the previous head (bs_amd/ab/libbsgpu_head.so: first-touch placement).
# The e2e and Writer legs with the process's CPUs on the far node (taskset, before any GPU use)
# and unpinned, alternated; then the host-copy and Writer tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for n in 0 1; do echo "node$n: $(cat /sys/devices/system/node/node$n/cpulist)"; done > gpurun_out/r06_c9_nodes.txt
FAR=$(cat /sys/devices/system/node/node1/cpulist)
LEGS="--steps 5 --warmup 2 --configs2-steps 0 --cpu-sample-mib 0"
for i in 1 2 3; do
  BSG_LIB_PATH=bs_amd/ab/libbsgpu_head.so timeout -k 10 200 taskset -c $FAR python -u bench.py $LEGS > gpurun_out/r06_c9_far_head_$i.log 2>&1 || exit $?
  timeout -k 10 200 taskset -c $FAR python -u bench.py $LEGS > gpurun_out/r06_c9_far_new_$i.log 2>&1 || exit $?
done
for i in 1 2; do
  BSG_LIB_PATH=bs_amd/ab/libbsgpu_head.so timeout -k 10 200 python -u bench.py $LEGS > gpurun_out/r06_c9_free_head_$i.log 2>&1 || exit $?
  timeout -k 10 200 python -u bench.py $LEGS > gpurun_out/r06_c9_free_new_$i.log 2>&1 || exit $?
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_host_copy.py tests/test_gpu_split_writer.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_c9_pytest.log 2>&1 || exit $?
