# Memory-latency counters of k_scan: in-flight VMEM / LDS instruction levels (level / count =
# average latency in cycles), plus TA/TCP busy.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS="--streams 16 --stream-mib 64 --steps 1 --warmup 0 --cpu-sample-mib 0 --e2e-mib 0"
timeout -s KILL 90 rocprofv3 --pmc SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/pmc_sq3 -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc_sq3.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum -d gpurun_out/pmc_sq4 -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc_sq4.log 2>&1
echo rc=$?
