# NUMA placement A/B (BSG_NUMA=1 vs the default 0): the Writer/raw A/B in unbound processes,
# N concurrent Writers, and the first-Writer costs, each with both settings.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L=bs_amd/libbsgpu.so
AB_ROUNDS=${AB_ROUNDS:-4} BSG_DEBUG_NUMA=1 timeout -k 10 400 python -u tools/writer_ab.py $L:BSG_NUMA=1 $L:BSG_NUMA=0 > gpurun_out/numa_writer_ab.log 2>&1 || exit $?
for v in 1 0; do
  BSG_NUMA=$v timeout -k 10 200 python -u tools/concurrent_writers.py > gpurun_out/numa_conc_$v.log 2>&1 || exit $?
done
for v in 1 0; do
  BSG_NUMA=$v timeout -k 10 200 python -u tools/first_writer.py first4g first4g first4g > gpurun_out/numa_first4g_$v.log 2>&1 || exit $?
done
