#!/bin/bash
# Builds a variant product library for an on-box A/B (tools/gpu/ab_lib.sh): the current sources with some files taken
# from a git revision. usage: tools/ab_build.sh <out.so> <rev> <file in zeebe_amd/csrc>...
set -e
out=$(realpath -m "$1"); rev=$2; shift 2
W=$(mktemp -d /tmp/abbuild.XXXX)
mkdir -p $W/zeebe_amd $W/include
cp -r zeebe_amd/csrc $W/zeebe_amd/csrc
rm -rf $W/zeebe_amd/csrc/build $W/zeebe_amd/csrc/build_checked $W/zeebe_amd/csrc/build_phases
cp include/*.h $W/include/
for f in "$@"; do git show $rev:zeebe_amd/csrc/$f > $W/zeebe_amd/csrc/$f; done
mkdir -p $(dirname $out)
make -s -C $W/zeebe_amd/csrc -j8 OUT=$out
rm -rf $W
