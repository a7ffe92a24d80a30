# k_scan memory-side counters on configs[2] (256 x 64 MiB): wave waits, VMEM in flight, TA busy,
# L2 hit/miss and EA read requests. One counter group per pass.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS="--streams 256 --stream-mib 64 --steps 1 --warmup 0 --cpu-sample-mib 0 --e2e-mib 0"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES -d gpurun_out/scanpmc_a -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/scanpmc_a.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum -d gpurun_out/scanpmc_b -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/scanpmc_b.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d gpurun_out/scanpmc_c -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/scanpmc_c.log 2>&1
