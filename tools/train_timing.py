"""Time the IPPO learner's phases on the GPU (rollout vs PPO epochs) at the metric config."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "jaxmarl-hft_amd")]

import torch  # noqa: E402

from hftlob.config_io import builtin_config  # noqa: E402
from hftlob.data.synthetic import generate_day  # noqa: E402
from hftlob.env import MARLEnv  # noqa: E402
from hftlob.train import ippo as I  # noqa: E402


def main():
    cfg = builtin_config("2_player_fq_fqc")
    w = cfg.world_config
    day = generate_day(n_msgs=100_000, seed=4, snap_every=w.n_data_msg_per_step * w.start_resolution)
    env = MARLEnv(None, cfg, data=day, return_info=False, persistent_outputs=True)
    graph = "--graph" in sys.argv
    c = I.default_config(NUM_ENVS=4096, NUM_STEPS=64, TOTAL_TIMESTEPS=4096 * 64 * 50, CUDA_GRAPHS=graph)
    tr = I.IPPOTrainer(env, c)
    tr.update()
    torch.cuda.synchronize()
    for _ in range(3):
        t0 = time.perf_counter()
        tr.rollout()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        tr.update()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"rollout {1e3 * (t1 - t0):.1f} ms  full update (rollout + epochs) {1e3 * (t2 - t1):.1f} ms  "
              f"-> {4096 * 64 / (t2 - t1):.0f} env-steps/s", flush=True)


if __name__ == "__main__":
    main()
