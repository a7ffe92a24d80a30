# SQ counters of k_scan (and the other kernels) on a scan-heavy run: 16 x 64 MiB streams.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS="--streams 16 --stream-mib 64 --steps 1 --warmup 0 --cpu-sample-mib 0"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS -d gpurun_out/pmc_sq1 -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc_sq1.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVES -d gpurun_out/pmc_sq2 -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc_sq2.log 2>&1
