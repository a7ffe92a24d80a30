# k_sha per-lane mode: register-message vs HBM-message ubench, and issue/wait counters of
# k_sha on configs[2] (two PMC passes of <= 8 SQ counters each).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/lanepmc
export TMPDIR=/tmp
timeout -k 10 60 tools/ubench/lanes_mem > gpurun_out/lanepmc/lanes_mem.log 2>&1 || exit $?
ARGS="--streams 256 --stream-mib 64 --steps 1 --warmup 0 --cpu-sample-mib 0 --e2e-mib 0"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_SALU -d gpurun_out/lanepmc/a -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/lanepmc/a.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_IFETCH SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_THREAD_CYCLES_VALU SQ_INSTS_SMEM SQ_WAVES -d gpurun_out/lanepmc/b -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/lanepmc/b.log 2>&1 || exit $?
echo done
