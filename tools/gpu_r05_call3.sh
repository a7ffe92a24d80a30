# Round 5, third GPU call: what made the new k_scan stage slower than round 4's (a same-box A/B of
# one-change variants on configs[2] alone, three interleaved rounds; stamps with and without the
# LDS stream cache), the prefix by blockIdx (parity: the suite's split tests), and the streaming
# path's host copy threads (BSG_COPY_THREADS 8 / 12 / 16, three processes each).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
python -m bs_amd.build
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_large_streams.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_pytest_call3.log 2>&1 || exit $?
BSG_LIB_PATH=bs_amd/variants/lib_diag.so timeout -k 10 200 python tools/scan_stamps.py > gpurun_out/r05_scan_stamps3.log 2>&1 || exit $?
BSG_LIB_PATH=bs_amd/variants/lib_diagnosc.so timeout -k 10 200 python tools/scan_stamps.py > gpurun_out/r05_scan_stamps3_nosc.log 2>&1 || exit $?
for r in 1 2 3; do
  for v in r4 new nosc noscwg load3 p3; do
    echo "== $v round $r" >> gpurun_out/r05_ab3.log
    if [ $v = new ]; then lib=bs_amd/libbsgpu.so; else lib=bs_amd/variants/lib_$v.so; fi
    BSG_LIB_PATH=$lib timeout -k 10 120 python bench.py --streams 256 --stream-mib 64 --steps 10 --warmup 3 --cpu-sample-mib 0 --e2e-mib 0 >> gpurun_out/r05_ab3.log 2>&1 || exit $?
  done
done
for r in 1 2 3; do
  for t in 8 12 16; do
    echo "== copy threads $t round $r" >> gpurun_out/r05_e2e_threads.log
    BSG_COPY_THREADS=$t E2E_REPS=6 timeout -k 10 120 python tools/e2e_trace_run.py >> gpurun_out/r05_e2e_threads.log 2>&1 || exit $?
  done
done
