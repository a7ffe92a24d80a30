# Round 5, fourteenth GPU call: k_scan strip pairs (BSG_SCAN_PAIR, the default library) against
# single strips (lib_nopair): the GPU suite, phase stamps, HBM read bytes by request size, then
# configs[2] and configs[1] A/B, three interleaved rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_pytest_gpu_call14.log 2>&1 || exit $?
BSG_LIB_PATH=bs_amd/variants/lib_diagpair.so timeout -k 10 200 python tools/scan_stamps.py > gpurun_out/r05_scan_stamps14_pair.log 2>&1 || exit $?
PMC="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
timeout -s KILL 200 rocprofv3 --pmc $PMC -d gpurun_out/rdreq14_c1 -o run --output-format csv -- python3 bench.py --cpu-sample-mib 0 --e2e-mib 0 --configs2-steps 0 --steps 1 --warmup 0 > gpurun_out/rdreq14_c1.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc $PMC -d gpurun_out/rdreq14_c2 -o run --output-format csv -- python3 bench.py --streams 256 --stream-mib 64 --cpu-sample-mib 0 --e2e-mib 0 --steps 1 --warmup 0 > gpurun_out/rdreq14_c2.log 2>&1 || exit $?
for r in 1 2 3; do
  for v in new nopair; do
    if [ $v = new ]; then lib=bs_amd/libbsgpu.so; else lib=bs_amd/variants/lib_$v.so; fi
    echo "== $v round $r" >> gpurun_out/r05_ab14_c2.log
    BSG_LIB_PATH=$lib timeout -k 10 120 python bench.py --streams 256 --stream-mib 64 --steps 10 --warmup 3 --cpu-sample-mib 0 --e2e-mib 0 >> gpurun_out/r05_ab14_c2.log 2>&1 || exit $?
    echo "== $v round $r" >> gpurun_out/r05_ab14_c1.log
    BSG_LIB_PATH=$lib timeout -k 10 120 python bench.py --steps 20 --warmup 5 --configs2-steps 0 --cpu-sample-mib 0 --e2e-mib 0 >> gpurun_out/r05_ab14_c1.log 2>&1 || exit $?
  done
done
