# Round 5, thirteenth GPU call: HBM read bytes by request size (TCC_EA0_RDREQ split into 32/64/128-B
# requests, one pass) for configs[1], configs[2] and the strip-pattern calibration, so the k_scan
# traffic ratio no longer rests on FETCH_SIZE's gfx950 halving of 128-B requests.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
PMC="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
timeout -s KILL 60 rocprofv3 --pmc $PMC -d gpurun_out/rdreq_calib -o run --output-format csv -- tools/ubench/scan_calib > gpurun_out/rdreq_calib.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc $PMC -d gpurun_out/rdreq_c1 -o run --output-format csv -- python3 bench.py --cpu-sample-mib 0 --e2e-mib 0 --configs2-steps 0 --steps 1 --warmup 0 > gpurun_out/rdreq_c1.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc $PMC -d gpurun_out/rdreq_c2 -o run --output-format csv -- python3 bench.py --streams 256 --stream-mib 64 --cpu-sample-mib 0 --e2e-mib 0 --steps 1 --warmup 0 > gpurun_out/rdreq_c2.log 2>&1
