#!/bin/bash
# rocprofv3 kernel stats of tools/train_timing.py (the IPPO learner at 4096 envs)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/ttp
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python $GRAFT_REPO_ROOT/tools/train_timing.py "$@" > $O/log.txt 2>&1
find $O -name "*kernel_trace.csv" -delete
