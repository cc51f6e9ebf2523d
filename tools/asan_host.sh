#!/bin/bash
# Host-side AddressSanitizer run (CPU only; GPU ASan is not available on this pool): builds
# libiris_asan.so with -fsanitize=address on the host code of every translation unit and
# runs the CPU test suite (JSON reader/writer, host query builders, ABI helpers) against it.
set -e -o pipefail
cd "$(dirname "$0")/.."
# the instrumented library is not left in the tree (gpurun would ship it with every call)
trap 'rm -f mpc-iris-code_amd/libiris_asan.so' EXIT
make -C mpc-iris-code_amd -j8 BUILD=build_asan LIB=libiris_asan.so \
    HIPFLAGS="-O1 -g -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer" \
    HOSTFLAGS="-O1 -g -std=c++17 -fPIC -Wall -fsanitize=address -fno-omit-frame-pointer -fno-gpu-sanitize"
RT=$(find /opt/rocm/lib/llvm/lib/clang -name "libclang_rt.asan-x86_64.so" | head -1)
IRIS_HIP_LIB=$PWD/mpc-iris-code_amd/libiris_asan.so LD_PRELOAD=$RT ASAN_OPTIONS=detect_leaks=0 \
    python -m pytest tests -q -m "not gpu" -p no:cacheprovider
