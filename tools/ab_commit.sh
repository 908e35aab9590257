#!/bin/bash
# Builds the product library of an earlier commit for an on-box A/B (tools/gpu/wave_ab.sh, tools/gpu/wave_prof.sh):
# the commit's zeebe_amd/csrc + include checked out into a scratch tree and built with that commit's own Makefile.
# usage: tools/ab_commit.sh <commit> [out.so]   (default out: ab/libzbgpu_<short sha>.so)
set -e
c=$(git rev-parse --short "$1")
out=$(realpath -m "${2:-ab/libzbgpu_$c.so}")
W=$(mktemp -d /tmp/abcommit.XXXX)
git archive "$c" zeebe_amd/csrc include | tar -x -C $W
rm -rf $W/zeebe_amd/csrc/build $W/zeebe_amd/csrc/build_checked $W/zeebe_amd/csrc/build_phases
mkdir -p $(dirname $out)
make -s -C $W/zeebe_amd/csrc -j${JOBS:-8} OUT=$out
rm -rf $W
echo "built $out"
