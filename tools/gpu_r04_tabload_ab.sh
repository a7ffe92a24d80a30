# k_scan / k_refine table load with all loads issued first (default) against the load-store loop
# (lib_prevtab): the -m gpu suite, kernel statistics of configs[1] and configs[2] per build, and
# bench lines, two interleaved rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tab
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04_pytest_gpu_tab.log 2>&1 || exit $?
for v in new prev; do
  L=""; [ $v = prev ] && L=bs_amd/variants/lib_prevtab.so
  BSG_LIB_PATH=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tab/$v -o run --output-format csv -- python3 bench.py --cpu-sample-mib 0 --e2e-mib 0 --steps 5 --warmup 2 > gpurun_out/tab/$v.log 2>&1 || exit $?
done
for r in 1 2; do
  for v in new prev; do
    L=""; [ $v = prev ] && L=bs_amd/variants/lib_prevtab.so
    echo "== $v round $r" >> gpurun_out/r04_tab_ab.log
    BSG_LIB_PATH=$L timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-sample-mib 0 --e2e-mib 0 >> gpurun_out/r04_tab_ab.log 2>&1 || exit $?
  done
done
