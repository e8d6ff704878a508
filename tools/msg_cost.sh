#!/bin/bash
# Per-message-kind SQ counters of the engine.  Usage: tools/msg_cost.sh TAG
set -o pipefail
T=${1:-x}
O=$GRAFT_REPO_ROOT/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_BRANCH --output-format csv -d $O/mc_$T -o mc -- python $GRAFT_REPO_ROOT/tools/msg_cost.py > $O/mc_$T.log 2>&1 || exit 1
python $GRAFT_REPO_ROOT/tools/msg_cost.py --report $O/mc_$T > $O/mc_$T.txt 2>&1
