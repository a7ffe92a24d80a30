# A/B on one box: the current libbsgpu.so against a reference build (libbsgpu_old.so, the
# previous commit's kernels), configs[2] and configs[1], twice each, interleaved; then the GPU
# parity tests of the split path on the current library.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
A="--cpu-sample-mib 0 --e2e-mib 0"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_params.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_parity.log 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 120 python bench.py --streams 256 --stream-mib 64 $A --steps 5 > gpurun_out/ab_new_c2_$r.log 2>&1 || exit $?
  BSG_LIB_PATH=$GRAFT_REPO_ROOT/bs_amd/libbsgpu_old.so timeout -k 10 120 python bench.py --streams 256 --stream-mib 64 $A --steps 5 > gpurun_out/ab_old_c2_$r.log 2>&1 || exit $?
  timeout -k 10 120 python bench.py $A > gpurun_out/ab_new_c1_$r.log 2>&1 || exit $?
  BSG_LIB_PATH=$GRAFT_REPO_ROOT/bs_amd/libbsgpu_old.so timeout -k 10 120 python bench.py $A > gpurun_out/ab_old_c1_$r.log 2>&1 || exit $?
done
