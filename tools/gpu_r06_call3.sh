# Round 6, third GPU call: (1) latency of the Writer's one tree-node hash batch (64 nodes of
# ~11.5 KB, Close's shape for 1 GiB); (2) configs[2] with the round-5 library against the cleaned
# one, alternated three times (the per-lane loop's registers moved in the cleanup); (3) the full
# bench line without and with bsg_init up front (the Writer leg's Close ran ~2.5 ms longer inside
# the bench than standalone).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
HS_N=64 HS_SIZE=11500 timeout -k 10 120 python -u tools/hasher_small_bench.py > gpurun_out/r06_c3_hasher.log 2>&1 || exit $?
C2="--steps 20 --warmup 5 --streams 256 --stream-mib 64 --e2e-mib 0 --no-writer-e2e --cpu-sample-mib 0"
for i in 1 2 3; do
  BSG_POLL=1 BSG_LIB_PATH=bs_amd/ab/libbsgpu_r05.so BSG_LIB_PARTIAL=1 timeout -k 10 200 python -u bench.py $C2 > gpurun_out/r06_c3_c2_old_$i.log 2>&1 || exit $?
  BSG_POLL=1 timeout -k 10 200 python -u bench.py $C2 > gpurun_out/r06_c3_c2_new_$i.log 2>&1 || exit $?
done
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r06_c3_bench_plain.log 2>&1 || exit $?
BSG_BENCH_INIT=1 timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r06_c3_bench_init.log 2>&1 || exit $?
