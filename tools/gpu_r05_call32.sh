# Round 5, thirty-second GPU call (the head, after BSG_LANE_UNI and BSG_LANE_LOADN): k_sha per-lane mode's instruction mix, configs[2] with every
# job in per-lane mode (BSG_LONG_MODE=off), two SQ counter passes (instruction counts by type;
# active / wait cycles by type), for tools/lane_mix.py.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS="--streams 256 --stream-mib 64 --cpu-sample-mib 0 --e2e-mib 0 --steps 1 --warmup 0"
BSG_LONG_MODE=off timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_INSTS_VMEM -d gpurun_out/lanemix32a -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/lanemix32a.log 2>&1 || exit $?
BSG_LONG_MODE=off timeout -s KILL 200 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_FLAT -d gpurun_out/lanemix32b -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/lanemix32b.log 2>&1
