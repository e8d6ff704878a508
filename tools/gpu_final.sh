#!/bin/bash
# Round-end validation on the GPU box: every -m gpu test (one process), the smoke, the driver's
# bench command (N=1, 20 steps), the same under torchrun with the RCCL process group (world 1:
# init, barrier and the max over ranks on the GPU), and the default bench line (128 steps + the
# CPU baseline).  Usage: tools/gpu_final.sh TAG
set -o pipefail
T=${1:-final}
O=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 2
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || exit 3
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_torchrun.json 2> $O/bench_torchrun.err || exit 4
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || exit 5
