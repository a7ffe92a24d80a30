# Round 5, eighteenth GPU call: k_scan prefetches the next strip's history and first lines
# (BSG_SCAN_PF, the default library) against no prefetch (lib_nopf): scan parity tests, phase
# stamps, then configs[2] and configs[1] A/B, three interleaved rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_large_streams.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_pytest_call18.log 2>&1 || exit $?
BSG_LIB_PATH=bs_amd/variants/lib_diagpf.so timeout -k 10 200 python tools/scan_stamps.py > gpurun_out/r05_scan_stamps18_pf.log 2>&1 || exit $?
for r in 1 2 3; do
  for v in new nopf; do
    if [ $v = new ]; then lib=bs_amd/libbsgpu.so; else lib=bs_amd/variants/lib_$v.so; fi
    echo "== $v round $r" >> gpurun_out/r05_ab18_c2.log
    BSG_LIB_PATH=$lib timeout -k 10 120 python bench.py --streams 256 --stream-mib 64 --steps 10 --warmup 3 --cpu-sample-mib 0 --e2e-mib 0 >> gpurun_out/r05_ab18_c2.log 2>&1 || exit $?
    echo "== $v round $r" >> gpurun_out/r05_ab18_c1.log
    BSG_LIB_PATH=$lib timeout -k 10 120 python bench.py --steps 20 --warmup 5 --configs2-steps 0 --cpu-sample-mib 0 --e2e-mib 0 >> gpurun_out/r05_ab18_c1.log 2>&1 || exit $?
  done
done
