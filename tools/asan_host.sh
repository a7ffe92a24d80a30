# Host-side AddressSanitizer run of the CPU test suite (no GPU): builds libbsgpu.so with the host
# code instrumented (-Xarch_host -fsanitize=address; device code unchanged) into /tmp/asan and runs
# `pytest -m "not gpu"` against it (BSG_LIB_PATH), including the corrupt-tree Reader fuzz of
# tests/test_reader_cpu.py. GPU sanitizers are not available on the GPU pool; this is host only.
set -eo pipefail
cd "$(dirname "$0")/.."
mkdir -p /tmp/asan
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -shared \
  -Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer -shared-libsan \
  -o /tmp/asan/libbsgpu.so bs_amd/csrc/bsgpu_kernels.hip bs_amd/csrc/bsgpu_host.cpp \
  bs_amd/csrc/bs_split.cpp bs_amd/csrc/bs_filestore.cpp
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
BSG_LIB_PATH=/tmp/asan/libbsgpu.so LD_PRELOAD=$RT ASAN_OPTIONS=detect_leaks=0 \
  python -m pytest tests -q -m "not gpu" -p no:cacheprovider
