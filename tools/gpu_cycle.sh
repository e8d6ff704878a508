#!/bin/bash
# One GPU iteration: parity tests -> bench -> phase stamps -> PMC pass.  Usage: tools/gpu_cycle.sh TAG
set -o pipefail
T=${1:-x}
O=$GRAFT_REPO_ROOT/gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests/test_gpu_book.py tests/test_gpu_env.py -x -q -p no:cacheprovider > $O/t_$T.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_$T.json 2> $O/bench_$T.err || exit 2
timeout -k 10 300 python tools/diag_stamps.py > $O/stamps_$T.txt 2>&1 || exit 3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY --output-format csv -d $O/pmc_$T -o pmc -- python $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 16 --warmup 4 --n-msgs 100000 > $O/pmc_$T.log 2>&1 || exit 4
