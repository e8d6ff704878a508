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


def test_learner_on_device_matches_numpy():
    """A recorded device rollout through the GPU learner: GAE and the PPO loss terms against the
    float64 numpy restatements of tests/test_ippo.py (ippo_rnn_JAXMARL.py:668-765) at rtol 1e-5,
    and one minibatch step (gradient, global-norm clip, Adam) against a float64 CPU copy of the
    network with the clip (optax clip_by_global_norm) and Adam (optax.adam, eps 1e-5) in numpy."""
    import copy
    from test_ippo import np_gae, np_ppo_loss
    cfg = builtin_config("2_player_fq_fqc")
    w = cfg.world_config
    day = generate_day(n_msgs=30_000, seed=4, snap_every=w.n_data_msg_per_step * w.start_resolution)
    env = MARLEnv(None, cfg, data=day, return_info=False, persistent_outputs=True)
    E, T, MB = 64, 12, 2
    c = I.default_config(NUM_ENVS=E, NUM_STEPS=T, GRU_HIDDEN_DIM=32, FC_DIM_SIZE=32, NUM_MINIBATCHES=MB,
                         UPDATE_EPOCHS=1, TOTAL_TIMESTEPS=E * T * 4, GAMMA=[0.99, 0.95], GAE_LAMBDA=[0.9, 0.95])
    tr = I.IPPOTrainer(env, c)
    for _ in range(3):                     # some episodes progress; rewards become non-trivial
        tr.update()
    h0 = [h.clone() for h in tr.h]
    tr.rollout()
    npy = lambda x: x.detach().double().cpu().numpy()  # noqa: E731
    for i, net in enumerate(tr.nets):
        b, n = tr.buf[i], tr.n_actors[i]
        with torch.no_grad():
            _, _, last_val = net.step(tr.h[i], tr.last_obs[i], tr.last_done[i])
            adv, tgt = I.calculate_gae(b.reward, b.value, b.global_done, last_val, c["GAMMA"][i], c["GAE_LAMBDA"][i])
        want_adv, want_tgt = np_gae(npy(b.reward), npy(b.value), npy(b.global_done), npy(last_val),
                                    c["GAMMA"][i], c["GAE_LAMBDA"][i])
        assert np.allclose(npy(adv), want_adv, rtol=1e-5, atol=1e-5), f"type {i}: GAE"
        assert np.allclose(npy(tgt), want_tgt, rtol=1e-5, atol=1e-5), f"type {i}: targets"
        idx = torch.randperm(n, device=tr.device, generator=torch.Generator(device=tr.device).manual_seed(i))[:n // MB]
        eps, vf, ent = c["CLIP_EPS"], c["VF_COEF"][i], c["ENT_COEF"][i]
        with torch.no_grad():
            logits, values = net(h0[i][idx], b.obs[:, idx], b.done[:, idx])
            out = I.ppo_loss(logits, values, b.action[:, idx], b.value[:, idx], b.log_prob[:, idx], adv[:, idx],
                             tgt[:, idx], eps, vf, ent)
        want = np_ppo_loss(npy(logits), npy(values), npy(b.action[:, idx]).astype(np.int64), npy(b.value[:, idx]),
                           npy(b.log_prob[:, idx]), npy(adv[:, idx]), npy(tgt[:, idx]), eps, vf, ent)
        assert np.allclose([float(x) for x in out[:4]], want, rtol=1e-5, atol=1e-6), f"type {i}: loss terms"
        # one minibatch step through the trainer (fresh Adam state) vs float64 on the CPU
        ref = copy.deepcopy(net).double().cpu()
        tr.opts[i] = torch.optim.Adam(net.parameters(), lr=c["LR"][i], eps=1e-5)
        st = tr._static(i, n, MB)
        st["h0"].copy_(h0[i]); st["adv"].copy_(adv); st["tgt"].copy_(tgt); st["idx"].copy_(idx)
        tr.opts[i].zero_grad(set_to_none=True)
        tr._mb_step(i)
        cpu = lambda x: x.detach().cpu()  # noqa: E731
        lg, vv = ref(cpu(h0[i][idx]).double(), cpu(b.obs[:, idx]).double(), cpu(b.done[:, idx]))
        loss = I.ppo_loss(lg, vv, cpu(b.action[:, idx]), cpu(b.value[:, idx]).double(), cpu(b.log_prob[:, idx]).double(),
                          cpu(adv[:, idx]).double(), cpu(tgt[:, idx]).double(), eps, vf, ent)[0]
        loss.backward()
        grads = [p.grad.numpy() for p in ref.parameters()]
        norm = np.sqrt(sum((g ** 2).sum() for g in grads))
        mx = c["MAX_GRAD_NORM"][i]
        scale = 1.0 if norm < mx else mx / norm
        lr = c["LR"][i]
        for (name, p_dev), p_ref, g in zip(net.named_parameters(), ref.parameters(), grads):
            g = g * scale
            m, v = 0.1 * g, 0.001 * g * g                         # first Adam step, b1 0.9, b2 0.999
            upd = lr * (m / 0.1) / (np.sqrt(v / 0.001) + 1e-5)
            want_p = p_ref.detach().numpy() - upd
            assert np.allclose(npy(p_dev), want_p, rtol=1e-5, atol=lr * 2e-3), f"type {i}: {name} after one step"


def test_trainer_update_over_rccl_world1():
    """The multi-rank learner path (gradient pmean through torch.distributed) on the RCCL backend
    ("nccl" on ROCm), world_size 1 on the box's one GPU: the update runs with the collective in
    it and matches a trainer without a process group (the pmean of one rank is the identity)."""
    import socket
    import torch.distributed as dist
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cfg = builtin_config("2_player_fq_fqc")
    w = cfg.world_config
    day = generate_day(n_msgs=30_000, seed=4, snap_every=w.n_data_msg_per_step * w.start_resolution)
    c = lambda: I.default_config(NUM_ENVS=64, NUM_STEPS=8, GRU_HIDDEN_DIM=16, FC_DIM_SIZE=16,  # noqa: E731
                                 NUM_MINIBATCHES=2, UPDATE_EPOCHS=1, TOTAL_TIMESTEPS=64 * 8 * 4)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        # the bucketed all-reduce itself runs over RCCL (the trainer skips it at world_size 1)
        g = torch.nn.Parameter(torch.zeros(5, device="cuda"))
        g.grad = torch.arange(5, dtype=torch.float32, device="cuda")
        I._average_grads([g], dist)
        torch.cuda.synchronize()
        assert torch.equal(g.grad, torch.arange(5, dtype=torch.float32, device="cuda"))
        env1 = MARLEnv(None, cfg, data=day, return_info=False, persistent_outputs=True)
        tr1 = I.IPPOTrainer(env1, c(), dist=dist)
        tr1.update()
        torch.cuda.synchronize()
    finally:
        dist.destroy_process_group()
    env0 = MARLEnv(None, cfg, data=day, return_info=False, persistent_outputs=True)
    tr0 = I.IPPOTrainer(env0, c())
    tr0.update()
    for n1, n0 in zip(tr1.nets, tr0.nets):
        for a, b in zip(n1.parameters(), n0.parameters()):
            assert torch.allclose(a, b, rtol=1e-5, atol=1e-6)
