#!/bin/bash
# Where the time goes: the SQ instruction-count pass of the metric bench and the phase-stamp /
# in-kernel-clock diagnostic (ab/stamps.so, a -DHFTLOB_STAMPS build).  Usage: tools/gpu_diag.sh TAG
set -o pipefail
T=${1:-diag}
O=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $O
cd $GRAFT_REPO_ROOT
if [ -f ab/stamps.so ]; then
  HFTLOB_STAMPS_LIB=$GRAFT_REPO_ROOT/ab/stamps.so timeout -k 10 300 python tools/diag_stamps.py > $O/stamps.txt 2>&1 || exit 1
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_BRANCH --output-format csv -d $O/sq -o run -- python $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 32 --warmup 4 > $O/sq.log 2>&1 || exit 2
timeout -k 10 400 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_INSTS_MISC --output-format csv -d $O/lds -o run -- python $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 32 --warmup 4 > $O/lds.log 2>&1 || exit 3
python $GRAFT_REPO_ROOT/tools/summarize_profiles.py $O > $O/summary.txt 2>&1
