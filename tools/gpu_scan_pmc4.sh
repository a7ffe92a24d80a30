# k_scan issue/wait counters on configs[2] (two PMC passes).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/scanpmc
export TMPDIR=/tmp
ARGS="--streams 256 --stream-mib 64 --steps 1 --warmup 0 --cpu-sample-mib 0 --e2e-mib 0"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS -d gpurun_out/scanpmc/a -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/scanpmc/a.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_INSTS_SALU SQ_WAVES SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE -d gpurun_out/scanpmc/b -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/scanpmc/b.log 2>&1 || exit $?
echo done
