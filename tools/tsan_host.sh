# Host-side ThreadSanitizer run (twin of tools/asan_host.sh): builds libbsgpu.so with the host
# code instrumented (-Xarch_host -fsanitize=thread; device code unchanged) into /tmp/tsan, plus
# tools/tsan/stress.cpp, and runs the stress driver. Mode "cpu" (default) needs no GPU: store/file
# write groups with a failing blob, store/mem aliased Puts / Seal / Delete, concurrent Readers,
# the shared copy pool. Mode "gpu" (on the MI355X box) runs 8 split::Writers, a raw context and
# 8 verifying Readers at once. GPU sanitizers are not available on the pool; this is host only.
#   bash tools/tsan_host.sh [cpu|gpu|all]
set -eo pipefail
cd "$(dirname "$0")/.."
MODE=${1:-cpu}
OUT=${TSAN_OUT:-/tmp/tsan}
mkdir -p "$OUT"
HIPCC=/opt/rocm/bin/hipcc
if [ ! -f "$OUT/libbsgpu.so" ] || [ -n "$(find bs_amd/csrc include -newer "$OUT/libbsgpu.so" -type f)" ]; then
  $HIPCC --offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -shared \
    -Xarch_host -fsanitize=thread -Xarch_host -fno-omit-frame-pointer \
    -o "$OUT/libbsgpu.so" bs_amd/csrc/bsgpu_kernels.hip bs_amd/csrc/bsgpu_host.cpp \
    bs_amd/csrc/bs_split.cpp bs_amd/csrc/bs_filestore.cpp
fi
/opt/rocm/lib/llvm/bin/clang++ -O1 -g -std=c++17 -fsanitize=thread -fno-omit-frame-pointer \
  -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include tools/tsan/stress.cpp \
  -L"$OUT" -lbsgpu -Wl,-rpath,"$OUT" -o "$OUT/stress"
TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1 suppressions=$PWD/tools/tsan/suppressions.txt ${TSAN_OPTIONS:-}" "$OUT/stress" "$MODE"
