#!/bin/bash
# Builds a variant product library for an on-box A/B (tools/gpu/wave_ab.sh, tools/gpu/ab_lib.sh): the current sources
# compiled with extra -D switches of a measurement experiment (ZB_EXP_*, never set in the product build).
# usage: tools/ab_variant.sh <out.so> -DZB_EXP_...
set -e
out=$(realpath -m "$1"); shift
W=$(mktemp -d /tmp/abvar.XXXX)
mkdir -p $W/zeebe_amd $W/include
cp -r zeebe_amd/csrc $W/zeebe_amd/csrc
rm -rf $W/zeebe_amd/csrc/build $W/zeebe_amd/csrc/build_checked $W/zeebe_amd/csrc/build_phases
cp include/*.h $W/include/
mkdir -p $(dirname $out)
make -s -C $W/zeebe_amd/csrc -j8 OUT=$out FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-unused-variable $*"
rm -rf $W
