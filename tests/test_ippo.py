"""IPPO learner (hftlob.train.ippo): the math against numpy restatements of
ippo_rnn_JAXMARL.py (GAE :668-690, loss :718-765, LR schedule :503-509), the GRU
reset semantics of ScannedRNN (:53-78), full updates on a CPU stand-in env, and
the gradient pmean over two gloo ranks (ippo_rnn_JAXMARL_pmap.py:566-567)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from hftlob.train import ippo as I

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def np_gae(r, v, d, last, gamma, lam):
    """_calculate_gae / _get_advantages (:668-690) in float64: (advantages, targets)."""
    T, B = r.shape
    adv = np.zeros((T, B), np.float64)
    gae, nv = np.zeros(B), np.asarray(last, np.float64)
    for t in reversed(range(T)):          # reverse scan carrying (gae, next_value)
        delta = r[t] + gamma * nv * (1 - d[t]) - v[t]
        gae = delta + gamma * lam * (1 - d[t]) * gae
        adv[t] = gae
        nv = v[t].astype(np.float64)
    return adv, adv + v


def np_ppo_loss(logits, values, act, old_v, old_lp, gae, targets, eps, vf, ent):
    """_loss_fn (:718-765) in float64: (total, value_loss, actor_loss, entropy)."""
    logits, values, old_v, old_lp, gae, targets = (np.asarray(x, np.float64) for x in
                                                   (logits, values, old_v, old_lp, gae, targets))
    lp_all = logits - logits.max(-1, keepdims=True)
    lp_all = lp_all - np.log(np.exp(lp_all).sum(-1, keepdims=True))
    lp = np.take_along_axis(lp_all, np.asarray(act)[..., None], -1)[..., 0]
    vpc = old_v + np.clip(values - old_v, -eps, eps)
    vloss = 0.5 * np.maximum((values - targets) ** 2, (vpc - targets) ** 2).mean()
    ratio = np.exp(lp - old_lp)
    g = (gae - gae.mean()) / (gae.std() + 1e-8)
    aloss = -np.minimum(ratio * g, np.clip(ratio, 1 - eps, 1 + eps) * g).mean()
    entropy = -(np.exp(lp_all) * lp_all).sum(-1).mean()
    return aloss + vf * vloss - ent * entropy, vloss, aloss, entropy


def test_gae_matches_reference_formula():
    rng = np.random.default_rng(0)
    T, B = 9, 5
    r, v = rng.normal(size=(T, B)).astype(np.float32), rng.normal(size=(T, B)).astype(np.float32)
    d = rng.random((T, B)) < 0.2
    last = rng.normal(size=B).astype(np.float32)
    gamma, lam = 0.99, 0.9
    adv, _ = np_gae(r, v, d, last, gamma, lam)
    a, tg = I.calculate_gae(torch.from_numpy(r), torch.from_numpy(v), torch.from_numpy(d), torch.from_numpy(last),
                            gamma, lam)
    assert np.allclose(a.numpy(), adv, atol=1e-5) and np.allclose(tg.numpy(), adv + v, atol=1e-5)


def test_ppo_loss_matches_reference_formula():
    rng = np.random.default_rng(1)
    T, B, A = 4, 6, 3
    logits = rng.normal(size=(T, B, A)).astype(np.float32)
    values = rng.normal(size=(T, B)).astype(np.float32)
    act = rng.integers(0, A, (T, B))
    old_v, old_lp = rng.normal(size=(T, B)).astype(np.float32), -rng.random((T, B)).astype(np.float32)
    gae, targets = rng.normal(size=(T, B)).astype(np.float32), rng.normal(size=(T, B)).astype(np.float32)
    eps, vf, ent = 0.2, 0.5, 0.01
    total, vloss, aloss, entropy = np_ppo_loss(logits, values, act, old_v, old_lp, gae, targets, eps, vf, ent)
    out = I.ppo_loss(*(torch.from_numpy(x) for x in (logits, values, act, old_v, old_lp, gae, targets)), eps, vf, ent)
    assert np.allclose([float(x) for x in out[:4]], [total, vloss, aloss, entropy], rtol=1e-5, atol=1e-6)


def test_linear_schedule():
    assert I.linear_schedule(1.0, 0, 4, 4, 10) == 1.0
    assert I.linear_schedule(1.0, 15, 4, 4, 10) == 1.0          # count // 16 = 0
    assert I.linear_schedule(1.0, 16, 4, 4, 10) == pytest.approx(0.9)
    assert I.linear_schedule(2.0, 16 * 5, 4, 4, 10) == pytest.approx(1.0)


def test_gru_reset_on_done():
    torch.manual_seed(0)
    net = I.ActorCriticRNN(5, 4, 16, 8)
    obs = torch.randn(3, 5)
    h = torch.randn(3, 8)
    done = torch.tensor([True, False, True])
    h1, lg1, v1 = net.step(h, obs, done)
    h0, lg0, v0 = net.step(torch.zeros(3, 8), obs, torch.zeros(3, dtype=torch.bool))
    assert torch.allclose(h1[done], h0[done]) and not torch.allclose(h1[1], h0[1])
    assert lg1.shape == (3, 4) and v1.shape == (3,)


class _Space:
    def __init__(self, n=None, shape=None):
        self.n, self.shape = n, shape


class _MAC:
    number_of_agents_per_type = [1, 2]


class FakeEnv:
    """CPU stand-in with MARLEnv's interface: type 0 earns +1 for action 0; episodes end every 5 steps."""
    device = torch.device("cpu")
    list_of_agents_configs = [object(), object()]
    multi_agent_config = _MAC()
    observation_spaces = [_Space(shape=(3,)), _Space(shape=(4,))]
    action_spaces = [_Space(n=3), _Space(n=2)]
    default_params = None

    def split_keys(self, keys, n):
        k = keys.to(torch.int64)
        j = torch.arange(n, dtype=torch.int64)
        return ((k[:, None, :] * 1_000_003 + j[None, :, None] * 7919 + 17) % (2 ** 31)).to(torch.int32)

    def reset(self, keys, params):
        E = keys.shape[0]
        self.t = torch.zeros(E, dtype=torch.int64)
        return [torch.zeros(E, 1, 3), torch.zeros(E, 2, 4)], None

    def step(self, keys, state, actions, params):
        E = keys.shape[0]
        self.t += 1
        done = self.t % 5 == 0
        r0 = (actions[0].view(E, 1) == 0).float()
        obs = [torch.randn(E, 1, 3), torch.randn(E, 2, 4)]
        dones = {"__all__": done, "agents": [done[:, None], done[:, None].repeat(1, 2)]}
        return obs, state, [r0, torch.zeros(E, 2)], dones, {}


def test_updates_learn_on_fake_env():
    env = FakeEnv()
    c = I.default_config(NUM_ENVS=16, NUM_STEPS=10, GRU_HIDDEN_DIM=16, FC_DIM_SIZE=16, NUM_MINIBATCHES=2,
                         UPDATE_EPOCHS=2, TOTAL_TIMESTEPS=16 * 10 * 40, LR=[3e-3, 3e-3], SEED=0)
    tr = I.IPPOTrainer(env, c)
    before = [p.detach().clone() for p in tr.nets[0].parameters()]
    rewards = []
    for _ in range(40):
        m = tr.update()
        rewards.append(float(m["avg_reward"][0]))
        assert all(np.isfinite(float(v)) for d in m["loss"] for v in d.values())
    assert any(not torch.equal(a, b) for a, b in zip(before, tr.nets[0].parameters()))
    assert np.mean(rewards[-5:]) > np.mean(rewards[:5]) + 0.1      # learns to pick action 0
    assert tr.buf[1].obs.shape == (10, 32, 4) and tr.buf[0].action.shape == (10, 16)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "jaxmarl-hft_amd")]
    import torch.distributed as dist
    from hftlob.train import ippo as I2
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    p = torch.nn.Parameter(torch.zeros(3))
    p.grad = torch.full((3,), float(rank + 1))
    w = torch.nn.Parameter(torch.zeros(2, 2))
    w.grad = torch.full((2, 2), 10.0 * rank)
    I2._average_grads([p, w], dist)
    if rank == 0:
        q.put((p.grad.tolist(), w.grad.tolist()))
    dist.destroy_process_group()


def test_grad_pmean_two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(i, 2, port, q)) for i in range(2)]
    for p in procs:
        p.start()
    pg, wg = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert pg == [1.5, 1.5, 1.5] and wg == [[5.0, 5.0], [5.0, 5.0]]


def _shard_worker(rank, world, port, q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "jaxmarl-hft_amd"), os.path.join(ROOT, "tests")]
    import torch.distributed as dist
    from hftlob.train import ippo as I2
    from test_ippo import FakeEnv as FE
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    c = I2.default_config(NUM_ENVS=32, NUM_STEPS=4, GRU_HIDDEN_DIM=8, FC_DIM_SIZE=8, NUM_MINIBATCHES=2,
                          UPDATE_EPOCHS=1, TOTAL_TIMESTEPS=32 * 4 * 10, SEED=3)
    tr = I2.IPPOTrainer(FE(), c, dist=dist)
    tr.update()
    q.put((rank, tr.E, tr.num_updates, tr.reset_keys.tolist(), tr.buf[1].obs.shape[1]))
    dist.destroy_process_group()


def test_num_envs_is_global_over_ranks():
    """NUM_ENVS is the global env count (ippo_rnn_JAXMARL_pmap.py:209-211, 329): 2 ranks step 16
    envs each, NUM_UPDATES = TOTAL // NUM_STEPS // NUM_ENVS, and the ranks' reset keys are the
    two halves of one split(_rng, NUM_ENVS)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_shard_worker, args=(i, 2, port, q)) for i in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    env = FakeEnv()
    c = I.default_config(NUM_ENVS=32, NUM_STEPS=4, GRU_HIDDEN_DIM=8, FC_DIM_SIZE=8, NUM_MINIBATCHES=2,
                         UPDATE_EPOCHS=1, TOTAL_TIMESTEPS=32 * 4 * 10, SEED=3)
    single = I.IPPOTrainer(env, c)                     # 1 rank: all 32 envs, the same global keys
    assert single.E == 32 and single.num_updates == 10
    for rank, E, nu, keys, actors in res:
        assert (E, nu, actors) == (16, 10, 32)        # type 1 has 2 agents per env
        assert keys == single.reset_keys[16 * rank:16 * (rank + 1)].tolist()
    with pytest.raises(ValueError, match="multiple of the world size"):
        class _D:
            get_world_size = staticmethod(lambda: 3)
            get_rank = staticmethod(lambda: 0)
        I.IPPOTrainer(env, c, dist=_D())
