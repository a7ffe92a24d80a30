# Round 6, fifth GPU call: the solo octet loop (sha256_blocks_oct_solo: 560 instructions per
# block against 570) — the ubench's state check against the single-lane rounds and its cycles,
# its PMC beside the general loop's, the whole GPU suite, configs[1] against the round-5 library
# alternated three times, and a kernel trace of the Writer leg (the tree-node hash's 3 ms).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 ./tools/ubench/oct > gpurun_out/r06_c5_oct.log 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY -d gpurun_out/r06_oct_solo_pmc -o run --output-format csv -- ./tools/ubench/oct_pmc > gpurun_out/r06_c5_oct_pmc.log 2>&1 || exit $?
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06_c5_pytest.log 2>&1 || exit $?
C1="--steps 20 --warmup 5 --configs2-steps 0 --e2e-mib 0 --no-writer-e2e --cpu-sample-mib 0"
for i in 1 2 3; do
  BSG_POLL=1 BSG_LIB_PATH=bs_amd/ab/libbsgpu_r05.so BSG_LIB_PARTIAL=1 timeout -k 10 120 python -u bench.py $C1 > gpurun_out/r06_c5_c1_old_$i.log 2>&1 || exit $?
  BSG_POLL=1 timeout -k 10 120 python -u bench.py $C1 > gpurun_out/r06_c5_c1_new_$i.log 2>&1 || exit $?
done
WRITER_MIB=1024 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r06_writer_trace -o run --output-format csv -- python3 tools/writer_bench.py > gpurun_out/r06_c5_writer_trace.log 2>&1 || exit $?
