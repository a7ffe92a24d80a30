# k_scan HBM read traffic and time per strip size: for the default library
# and each variant (AB_VARIANTS): split-path parity tests, configs[1] / configs[2] bench lines
# (stage times) and a rocprofv3 FETCH_SIZE pass on configs[1].
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/scan_ab
export TMPDIR=/tmp
for lib in bs_amd/libbsgpu.so ${AB_VARIANTS}; do
  tag=$(basename $lib .so)
  export BSG_LIB_PATH=$PWD/$lib BSG_LIB_PARTIAL=1
  if [ "$lib" != bs_amd/libbsgpu.so ]; then
    timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py > gpurun_out/scan_ab/pytest_$tag.log 2>&1 || exit $?
  fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-sample-mib 0 --e2e-mib 0 --configs2-steps 10 > gpurun_out/scan_ab/bench_$tag.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/scan_ab/fetch_$tag -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --cpu-sample-mib 0 --e2e-mib 0 --configs2-steps 1 > gpurun_out/scan_ab/fetch_$tag.log 2>&1 || exit $?
done
