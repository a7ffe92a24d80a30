# Round 6, fourth GPU call: configs[2] with the round-5 library against the cleaned one after
# reg_head's form was restored (the per-lane loop compiles to round 5's layout again), three
# alternations; then the GPU tests that cover the per-lane regions and the early chains.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
C2="--steps 20 --warmup 5 --streams 256 --stream-mib 64 --e2e-mib 0 --no-writer-e2e --cpu-sample-mib 0"
for i in 1 2 3; do
  BSG_POLL=1 BSG_LIB_PATH=bs_amd/ab/libbsgpu_r05.so BSG_LIB_PARTIAL=1 timeout -k 10 200 python -u bench.py $C2 > gpurun_out/r06_c4_c2_old_$i.log 2>&1 || exit $?
  BSG_POLL=1 timeout -k 10 200 python -u bench.py $C2 > gpurun_out/r06_c4_c2_new_$i.log 2>&1 || exit $?
done
timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_host_copy.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_c4_pytest.log 2>&1 || exit $?
# e2e + Writer legs without and with bsg_init up front, alternated (configs[1] short, no configs[2])
LEGS="--steps 5 --warmup 2 --configs2-steps 0 --cpu-sample-mib 0"
for i in 1 2 3; do
  BSG_DEBUG_HASHER=1 timeout -k 10 200 python -u bench.py $LEGS > gpurun_out/r06_c4_legs_plain_$i.log 2>&1 || exit $?
  BSG_DEBUG_HASHER=1 BSG_BENCH_INIT=1 timeout -k 10 200 python -u bench.py $LEGS > gpurun_out/r06_c4_legs_init_$i.log 2>&1 || exit $?
done
# the octet chain alone (tools/ubench/oct_pmc: one lone wave, 4,000 blocks x 3 launches): its
# instruction mix and issue cycles, for DESIGN §4.1's account of the chain's last 7 %
./tools/ubench/oct_pmc > gpurun_out/r06_c4_oct_pmc_plain.log 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY -d gpurun_out/r06_oct_pmc -o run --output-format csv -- ./tools/ubench/oct_pmc > gpurun_out/r06_c4_oct_pmc.log 2>&1 || exit $?
