# Round 5, seventh GPU call: the aligned chain loops (octet and pair, K+W quads four at a time)
# in the product: the whole GPU suite, then bench lines A/B against the library before them
# (lib_prechain) and round 4 (lib_r4), two interleaved rounds of the default bench form.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 60 tools/ubench/oct_var > gpurun_out/r05_oct_var3.log 2>&1 || exit $?
python -m bs_amd.build
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_pytest_gpu_call7.log 2>&1 || exit $?
for r in 1 2; do
  for v in new prechain r4; do
    if [ $v = new ]; then lib=bs_amd/libbsgpu.so; else lib=bs_amd/variants/lib_$v.so; fi
    echo "== $v round $r" >> gpurun_out/r05_ab7.log
    BSG_LIB_PATH=$lib timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-sample-mib 0 --e2e-mib 0 >> gpurun_out/r05_ab7.log 2>&1 || exit $?
  done
done
