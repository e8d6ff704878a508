# A/B of MARLEnv.rollout_sampled env slices (bench.py --slices) on one GPU.
set -o pipefail
mkdir -p gpurun_out/sweep
timeout -k 10 300 python -u -m pytest tests/test_gpu_env.py -k "rollout_sampled" -x -q --timeout 120 --timeout-method thread > gpurun_out/sweep/tests.log 2>&1 || exit 3
for G in 2 3 4; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 128 --slices $G > gpurun_out/sweep/G$G.json 2> gpurun_out/sweep/G$G.err || exit 4
done
timeout -k 10 120 python bench.py --no-cpu-baseline --steps 512 --slices 2 > gpurun_out/sweep/G2_512.json 2> gpurun_out/sweep/G2_512.err || exit 5
