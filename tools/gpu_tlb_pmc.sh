# Address-translation counters (UTCL1) for the per-lane SHA ubench patterns and for k_sha on
# configs[2] with the default library and the round-2 per-lane variant (bs_amd/variants).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tlb
export TMPDIR=/tmp
C="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_SERIALIZATION_STALL_sum"
timeout -s KILL 90 rocprofv3 --pmc $C -d gpurun_out/tlb/ub -o run --output-format csv -- tools/ubench/lanes_mem > gpurun_out/tlb/ub.log 2>&1 || exit $?
ARGS="--streams 256 --stream-mib 64 --steps 1 --warmup 0 --cpu-sample-mib 0 --e2e-mib 0"
timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/tlb/new -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/tlb/new.log 2>&1 || exit $?
BSG_LIB_PATH=$PWD/bs_amd/variants/lib_oldlane.so timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/tlb/old -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/tlb/old.log 2>&1 || exit $?
echo done
