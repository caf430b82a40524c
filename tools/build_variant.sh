#!/bin/bash
# A/B variant of the engine library (CPU side, before a gpurun A/B): the same sources built with
# extra defines into kmerlsh_amd/lib_diag/libklsh_<name>.so (KLSH_LIB=... selects it at run time).
#   tools/build_variant.sh <name> "-DFOO=1 -DBAR"
set -e
cd "$(dirname "$0")/../kmerlsh_amd/csrc"
name=$1; shift
mkdir -p ../lib_diag ../build_ab/$name
make -s -j8 lib OBJDIR=../build_ab/$name LIB=../lib_diag/libklsh_$name.so EXTRA="$*"
echo "built kmerlsh_amd/lib_diag/libklsh_$name.so ($*)"
