#!/bin/bash
# Round-5 extras on the GPU box: the 2-rank same-device rehearsal of the N-GPU body (gloo) and
# the wave-time tail statistics of the final kernel at the driver's and the profile's launch
# lengths (needs ab/wavetime.so: make -C jaxmarl-hft_amd/csrc wavetime).  Usage: tools/gpu_extra.sh TAG
set -o pipefail
T=${1:-extra}
O=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --same-device --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_2rank_samedev_gloo.json 2> $O/bench_2rank.err || exit 1
WT_STEPS=20 timeout -k 10 300 python tools/diag_wavetime.py > $O/wavetime_20step.json 2> $O/wavetime.err || exit 2
WT_STEPS=128 timeout -k 10 300 python tools/diag_wavetime.py > $O/wavetime_128step.json 2>> $O/wavetime.err || exit 3
