# Round 5, twentieth GPU call: chained strips with the loop kept line-aligned in k_scan (BSG_SCAN_CHAIN=1, lib_chain: no history
# block read, the predecessor lane checks positions 0..62) against the default library: the whole
# GPU suite on lib_chain, its phase stamps and HBM read bytes by request size, then configs[2] and
# configs[1] A/B, three interleaved rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
BSG_LIB_PATH=bs_amd/variants/lib_chain.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_pytest_gpu_call20.log 2>&1 || exit $?
BSG_LIB_PATH=bs_amd/variants/lib_diagchain.so timeout -k 10 200 python tools/scan_stamps.py > gpurun_out/r05_scan_stamps20_chain.log 2>&1 || exit $?
PMC="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
BSG_LIB_PATH=bs_amd/variants/lib_chain.so timeout -s KILL 200 rocprofv3 --pmc $PMC -d gpurun_out/rdreq20_c1 -o run --output-format csv -- python3 bench.py --cpu-sample-mib 0 --e2e-mib 0 --configs2-steps 0 --steps 1 --warmup 0 > gpurun_out/rdreq20_c1.log 2>&1 || exit $?
BSG_LIB_PATH=bs_amd/variants/lib_chain.so timeout -s KILL 200 rocprofv3 --pmc $PMC -d gpurun_out/rdreq20_c2 -o run --output-format csv -- python3 bench.py --streams 256 --stream-mib 64 --cpu-sample-mib 0 --e2e-mib 0 --steps 1 --warmup 0 > gpurun_out/rdreq20_c2.log 2>&1 || exit $?
for r in 1 2 3; do
  for v in new chain; do
    if [ $v = new ]; then lib=bs_amd/libbsgpu.so; else lib=bs_amd/variants/lib_$v.so; fi
    echo "== $v round $r" >> gpurun_out/r05_ab20_c2.log
    BSG_LIB_PATH=$lib timeout -k 10 120 python bench.py --streams 256 --stream-mib 64 --steps 10 --warmup 3 --cpu-sample-mib 0 --e2e-mib 0 >> gpurun_out/r05_ab20_c2.log 2>&1 || exit $?
    echo "== $v round $r" >> gpurun_out/r05_ab20_c1.log
    BSG_LIB_PATH=$lib timeout -k 10 120 python bench.py --steps 20 --warmup 5 --configs2-steps 0 --cpu-sample-mib 0 --e2e-mib 0 >> gpurun_out/r05_ab20_c1.log 2>&1 || exit $?
  done
done
