#!/bin/bash
# Per-message-kind SQ counters of the engine (3 PMC passes).  Usage: tools/msg_cost.sh TAG
set -o pipefail
T=${1:-x}
O=$GRAFT_REPO_ROOT/gpurun_out
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_BRANCH"
P2="SQ_WAVES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_IFETCH SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM"
P3="SQ_WAVES SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_REQ"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/mc_$T/p0 -o mc -- python $GRAFT_REPO_ROOT/tools/msg_cost.py > $O/mc_$T.log 2>&1 || exit 1
i=0
for P in "$P1"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $O/mc_$T/p$i -o mc -- python $GRAFT_REPO_ROOT/tools/msg_cost.py > $O/mc_$T.log 2>&1 || exit 1
done
python $GRAFT_REPO_ROOT/tools/msg_cost.py --report $O/mc_$T > $O/mc_$T.txt 2>&1
