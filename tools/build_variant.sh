#!/bin/bash
# Build a diagnostic variant of libhftlob.so from the working tree into ab/lib_<name>.so with extra
# compile flags (timing / knockout builds; see the HFTLOB_KO_* / HFTLOB_NO_* switches in hftlob.hip).
# Usage: tools/build_variant.sh NAME "-DFLAG ..."
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p $ROOT/ab
make -C $ROOT/jaxmarl-hft_amd/csrc -j8 VARIANT=_$1 "VFLAGS=$2" OUT=$ROOT/ab/lib_$1.so > /tmp/build_$1.log 2>&1 || { tail -20 /tmp/build_$1.log; exit 1; }
