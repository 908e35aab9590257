#!/bin/bash
# Builds a variant product library for an on-box A/B (tools/gpu/kernel_ab.sh, tools/gpu/ab_lib.sh): the current sources
# with a measurement experiment applied -- a patch under tools/variants/ (PATCH=..., applied to a copy: the product
# sources carry no experiment switches) and / or extra -D flags.
# usage: [PATCH=tools/variants/x.patch] tools/ab_variant.sh <out.so> [-D...]
set -e
out=$(realpath -m "$1"); shift
W=$(mktemp -d /tmp/abvar.XXXX)
mkdir -p $W/zeebe_amd $W/include
cp -r zeebe_amd/csrc $W/zeebe_amd/csrc
rm -rf $W/zeebe_amd/csrc/build $W/zeebe_amd/csrc/build_checked $W/zeebe_amd/csrc/build_phases
cp include/*.h $W/include/
if [ -n "$PATCH" ]; then patch -s -d $W/zeebe_amd/csrc -p1 < "$PATCH"; fi
mkdir -p $(dirname $out)
make -s -C $W/zeebe_amd/csrc -j8 OUT=$out FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-unused-variable $*"
rm -rf $W
