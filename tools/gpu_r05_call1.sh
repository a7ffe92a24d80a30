# Round 5, first GPU call: parity of the new scan (LDS stream cache, per-workgroup refine lists,
# fold64 warm-up) on the whole GPU suite, k_scan phase stamps (BSG_SCAN_DIAG build), then a
# same-box A/B of the round-4 library, the new one and the new one with one global refine list.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
python -m bs_amd.build
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_pytest_gpu_scan1.log 2>&1 || exit $?
BSG_LIB_PATH=bs_amd/variants/lib_diag.so timeout -k 10 200 python tools/scan_stamps.py > gpurun_out/r05_scan_stamps.log 2>&1 || exit $?
for r in 1 2; do
  for v in r4 new nowg; do
    echo "== $v round $r" >> gpurun_out/r05_scan_ab1.log
    if [ $v = new ]; then lib=bs_amd/libbsgpu.so; else lib=bs_amd/variants/lib_$v.so; fi
    BSG_LIB_PATH=$lib timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-sample-mib 0 --e2e-mib 0 >> gpurun_out/r05_scan_ab1.log 2>&1 || exit $?
  done
done
