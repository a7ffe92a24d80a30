# k_refine: exact-block lookups issued per group of 8 positions and 4 waves per SIMD (default)
# against the previous head (lib_prevtab): parity tests, kernel statistics of configs[1] and
# configs[2] per build, and bench lines, two interleaved rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/refine
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large_streams.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04_pytest_gpu_refine.log 2>&1 || exit $?
for v in new prev; do
  L=""; [ $v = prev ] && L=bs_amd/variants/lib_prevtab.so
  BSG_LIB_PATH=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/refine/$v -o run --output-format csv -- python3 bench.py --cpu-sample-mib 0 --e2e-mib 0 --steps 5 --warmup 2 > gpurun_out/refine/$v.log 2>&1 || exit $?
done
for r in 1 2; do
  for v in new prev; do
    L=""; [ $v = prev ] && L=bs_amd/variants/lib_prevtab.so
    echo "== $v round $r" >> gpurun_out/r04_refine_ab.log
    BSG_LIB_PATH=$L timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-sample-mib 0 --e2e-mib 0 >> gpurun_out/r04_refine_ab.log 2>&1 || exit $?
  done
done
