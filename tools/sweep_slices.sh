# A/B of MARLEnv.rollout_sampled launch shapes (bench.py --slices) on one GPU: 0 = one persistent
# k_env_rollout launch (every env's steps back to back), 1..4 = env slices on their own streams.
set -o pipefail
O=gpurun_out/${1:-sweep}
mkdir -p $O
for r in 1 2; do for G in 0 1 2 3 4; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 128 --slices $G > $O/G${G}_$r.json 2> $O/G$G.err || exit 4
done; done
