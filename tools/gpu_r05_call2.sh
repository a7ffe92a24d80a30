# Round 5, second GPU call: parity of the new prelude (LDS strip jobs, per-workgroup refine
# lists, single-pass prefix, chain-first schedule for light runs, k_pick before k_rescan) on the
# whole GPU suite; k_scan phase stamps; a same-box A/B against the round-4 library and one-change
# variants; the SQ counter passes for the work roofline (configs[2]) and the chain (k_early,
# configs[1], and the bare octet loop); one e2e rep traced with the HIP API and host stamps.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
python -m bs_amd.build
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_pytest_gpu_call2.log 2>&1 || exit $?
BSG_LIB_PATH=bs_amd/variants/lib_diag.so timeout -k 10 200 python tools/scan_stamps.py > gpurun_out/r05_scan_stamps2.log 2>&1 || exit $?
BSG_LIB_PATH=bs_amd/variants/lib_diag3.so timeout -k 10 200 python tools/scan_stamps.py > gpurun_out/r05_scan_stamps2_load3.log 2>&1 || exit $?
for r in 1 2; do
  for v in r4 new p3 load3 load3w nowg; do
    echo "== $v round $r" >> gpurun_out/r05_ab2.log
    if [ $v = new ]; then lib=bs_amd/libbsgpu.so; else lib=bs_amd/variants/lib_$v.so; fi
    BSG_LIB_PATH=$lib timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-sample-mib 0 --e2e-mib 0 >> gpurun_out/r05_ab2.log 2>&1 || exit $?
  done
done
timeout -k 10 60 rocprofv3 -L > gpurun_out/r05_counters_list.txt 2>&1 || true
CTRS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_IFETCH GRBM_GUI_ACTIVE"
timeout -s KILL 180 rocprofv3 --pmc $CTRS -d gpurun_out/pmc_c2 -o run --output-format csv -- python3 bench.py --streams 256 --stream-mib 64 --cpu-sample-mib 0 --e2e-mib 0 --steps 1 --warmup 1 > gpurun_out/pmc_c2.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc $CTRS -d gpurun_out/pmc_c1 -o run --output-format csv -- python3 bench.py --cpu-sample-mib 0 --e2e-mib 0 --configs2-steps 0 --steps 1 --warmup 1 > gpurun_out/pmc_c1.log 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --pmc $CTRS -d gpurun_out/pmc_oct -o run --output-format csv -- tools/ubench/oct_pmc > gpurun_out/pmc_oct.log 2>&1 || exit $?
OUT=r05_e2e_trace HIP_TRACE=1 bash tools/gpu_e2e_trace.sh
