cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in libbsgpu_v4.so; do
VARIANT=$v BSG_LONG_MODE=all timeout -k 5 20 python tools/repro_hang.py > gpurun_out/repro_$v.log 2>&1; echo "rc=$?" >> gpurun_out/repro_$v.log
done
