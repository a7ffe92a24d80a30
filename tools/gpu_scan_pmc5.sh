# k_scan (bench, configs[2], one step) against its replay (tools/ubench/scanload, k_full): wave
# waits, LDS issue and bank conflicts, VALU activity. One pass, 8 SQ counters.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"
timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/pmc5_bench -o run --output-format csv -- python3 bench.py --streams 256 --stream-mib 64 --steps 1 --warmup 1 --cpu-sample-mib 0 --e2e-mib 0 > gpurun_out/pmc5_bench.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/pmc5_replay -o run --output-format csv -- ./tools/ubench/scanload > gpurun_out/pmc5_replay.log 2>&1
