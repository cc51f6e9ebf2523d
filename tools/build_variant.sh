#!/bin/bash
# Builds a diagnostic / variant copy of the library: tools/build_variant.sh NAME "-DFLAG=.. ..."
# -> mpc-iris-code_amd/libiris_NAME.so (build dir build_NAME); never the shipped library.
set -e
name=$1; shift
make -C "$(dirname "$0")/../mpc-iris-code_amd" -j8 ARCH=gfx950 BUILD=build_$name LIB=libiris_$name.so \
    HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result $*" >/dev/null
echo "built libiris_$name.so ($*)"
