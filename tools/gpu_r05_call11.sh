# Round 5, eleventh GPU call: k_scan strip groups by ticket (BSG_SCAN_DYN, the default library)
# against the fixed stride (lib_scanstatic): parity of the scan tests, the GPU suite, k_scan phase
# stamps of the ticket form, then configs[2] and configs[1] A/B, three interleaved rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_pytest_gpu_call11.log 2>&1 || exit $?
BSG_LIB_PATH=bs_amd/variants/lib_diagdyn.so timeout -k 10 200 python tools/scan_stamps.py > gpurun_out/r05_scan_stamps11_dyn.log 2>&1 || exit $?
for r in 1 2 3; do
  for v in new scanstatic; do
    if [ $v = new ]; then lib=bs_amd/libbsgpu.so; else lib=bs_amd/variants/lib_$v.so; fi
    echo "== $v round $r" >> gpurun_out/r05_ab11_c2.log
    BSG_LIB_PATH=$lib timeout -k 10 120 python bench.py --streams 256 --stream-mib 64 --steps 10 --warmup 3 --cpu-sample-mib 0 --e2e-mib 0 >> gpurun_out/r05_ab11_c2.log 2>&1 || exit $?
    echo "== $v round $r" >> gpurun_out/r05_ab11_c1.log
    BSG_LIB_PATH=$lib timeout -k 10 120 python bench.py --steps 20 --warmup 5 --configs2-steps 0 --cpu-sample-mib 0 --e2e-mib 0 >> gpurun_out/r05_ab11_c1.log 2>&1 || exit $?
  done
done
