# Round 5, thirty-seventh GPU call: as the thirty-fifth, with the last three rounds of k_scan strip groups
# claimed just in time (kScanJitRounds 3; the first try, one round, claimed too late to matter):
# against tickets claimed two iterations ahead (lib_nojit): the scan-edge and parity GPU tests,
# per-wave stamps (a BSG_SCAN_DIAG build), then configs[1] and configs[2] A/B, three rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_scan_edges.py tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r05_pytest_jit37.log 2>&1 || exit $?
BSG_LIB_PATH=bs_amd/variants/lib_diag.so timeout -k 10 200 python tools/scan_stamps.py > gpurun_out/r05_scan_stamps37_jit.log 2>&1 || exit $?
for r in 1 2 3; do
  for v in jit nojit; do
    if [ $v = jit ]; then lib=bs_amd/libbsgpu.so; else lib=bs_amd/variants/lib_$v.so; fi
    echo "== $v round $r" >> gpurun_out/r05_ab37_c1.log
    BSG_LIB_PATH=$lib timeout -k 10 120 python bench.py --steps 20 --warmup 5 --configs2-steps 0 --cpu-sample-mib 0 --e2e-mib 0 >> gpurun_out/r05_ab37_c1.log 2>&1 || exit $?
    echo "== $v round $r" >> gpurun_out/r05_ab37_c2.log
    BSG_LIB_PATH=$lib timeout -k 10 120 python bench.py --streams 256 --stream-mib 64 --steps 10 --warmup 3 --cpu-sample-mib 0 --e2e-mib 0 >> gpurun_out/r05_ab37_c2.log 2>&1 || exit $?
  done
done
