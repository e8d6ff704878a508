#!/bin/bash
# Build libhftlob.so from a git revision (default HEAD) into ab/lib_<name>.so, for interleaved
# A/B runs against the working tree's build (tools/ab_quick.sh).  Usage: tools/build_prev.sh [REV] [NAME]
set -e
REV=${1:-HEAD}
NAME=${2:-prev}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d /tmp/hftlob_rev.XXXX)
mkdir -p $T/jaxmarl-hft_amd/csrc $T/include
git -C $ROOT show $REV:jaxmarl-hft_amd/csrc/hftlob.hip > $T/jaxmarl-hft_amd/csrc/hftlob.hip
git -C $ROOT show $REV:jaxmarl-hft_amd/csrc/Makefile > $T/jaxmarl-hft_amd/csrc/Makefile
git -C $ROOT show $REV:include/hftlob.h > $T/include/hftlob.h
mkdir -p $ROOT/ab
make -C $T/jaxmarl-hft_amd/csrc -j8 OUT=$ROOT/ab/lib_$NAME.so > $T/build.log 2>&1 || { tail -20 $T/build.log; exit 1; }
rm -rf $T
