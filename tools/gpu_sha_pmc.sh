# k_sha instruction-issue counters on configs[1] and configs[2] (one PMC group per pass).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in c1 c2; do
  if [ $cfg = c2 ]; then ARGS="--streams 256 --stream-mib 64"; else ARGS=""; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_IFETCH SQ_BUSY_CYCLES -d gpurun_out/shapmc_${cfg}_a -o run --output-format csv -- python3 bench.py $ARGS --steps 1 --warmup 0 --cpu-sample-mib 0 --e2e-mib 0 > gpurun_out/shapmc_${cfg}_a.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE -d gpurun_out/shapmc_${cfg}_b -o run --output-format csv -- python3 bench.py $ARGS --steps 1 --warmup 0 --cpu-sample-mib 0 --e2e-mib 0 > gpurun_out/shapmc_${cfg}_b.log 2>&1 || exit $?
done
