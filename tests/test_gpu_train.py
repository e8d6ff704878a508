"""IPPO learner on the HIP env (hftlob.train.ippo with MARLEnv): updates run with the
device rollout, losses stay finite, and the rollout buffers hold the env's outputs."""
import numpy as np
import pytest
import torch

from hftlob.config_io import builtin_config
from hftlob.data.synthetic import generate_day
from hftlob.env import MARLEnv, split_keys
from hftlob.train import ippo as I

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["2_player_fq_fqc", "3_player_fq_fqc_dir"])
def test_ippo_updates_on_hip_env(name):
    cfg = builtin_config(name)
    w = cfg.world_config
    day = generate_day(n_msgs=30_000, seed=4, snap_every=w.n_data_msg_per_step * w.start_resolution)
    env = MARLEnv(None, cfg, data=day, return_info=False, persistent_outputs=True)
    c = I.default_config(NUM_ENVS=128, NUM_STEPS=16, GRU_HIDDEN_DIM=32, FC_DIM_SIZE=32, NUM_MINIBATCHES=4,
                         UPDATE_EPOCHS=2, TOTAL_TIMESTEPS=128 * 16 * 4, NUM_AGENTS_PER_TYPE=cfg.number_of_agents_per_type)
    tr = I.IPPOTrainer(env, c)
    for _ in range(3):
        m = tr.update()
        for d in m["loss"]:
            assert all(np.isfinite(float(v)) for v in d.values())
    for i, b in enumerate(tr.buf):
        assert b.obs.shape[0] == 16 and b.obs.shape[1] == tr.n_actors[i]
        assert int(b.action.min()) >= 0 and int(b.action.max()) < env.action_spaces[i].n
        assert torch.isfinite(b.reward).all() and torch.isfinite(b.obs).all()
    # episodes of 64 steps: over 48 steps of 128 envs some auto-reset has happened only if the
    # windows start mid-episode; the env's own done bookkeeping is checked by tests/test_gpu_env.py


def test_graph_rollout_replays_the_env_exactly():
    """The HIP-graph rollout (3rd call: a replay) against eager env steps fed the actions it
    recorded: same rewards and next observations, bit for bit."""
    cfg = builtin_config("2_player_fq_fqc")
    w = cfg.world_config
    day = generate_day(n_msgs=30_000, seed=4, snap_every=w.n_data_msg_per_step * w.start_resolution)
    env = MARLEnv(None, cfg, data=day, return_info=False, persistent_outputs=True)
    E, T = 64, 8
    c = I.default_config(NUM_ENVS=E, NUM_STEPS=T, GRU_HIDDEN_DIM=32, FC_DIM_SIZE=32, TOTAL_TIMESTEPS=E * T * 4,
                         CUDA_GRAPHS=True)
    tr = I.IPPOTrainer(env, c)
    tr.rollout()
    tr.rollout()
    assert isinstance(tr._roll, torch.cuda.CUDAGraph)
    state0 = tr.state.clone(env)
    rng0 = tr.rng.clone()
    tr.rollout()                                   # a replay
    torch.cuda.synchronize()
    acts = [b.action.clone() for b in tr.buf]
    rews = [b.reward.clone() for b in tr.buf]
    obs_next = [b.obs.clone() for b in tr.buf]
    state, rng = state0, rng0
    for t in range(T):
        k = split_keys(rng[None], 2)[0]             # IPPOTrainer._next_keys
        rng = k[0].clone()
        keys = split_keys(k[1:2].contiguous(), E)[0].contiguous()
        obs, state, rew, dones, _ = env.step(keys, state, [a[t].view(E, -1) for a in acts], env.default_params)
        for i in range(len(acts)):
            assert torch.equal(rew[i].reshape(-1), rews[i][t]), (t, i)
            if t + 1 < T:
                assert torch.equal(obs[i].reshape(obs_next[i].shape[1], -1), obs_next[i][t + 1]), (t, i)
    assert torch.equal(state.buf, tr.state.buf)
