"""Fused env step parity: HIP hftlob_env_step vs the CPU oracle over episodes."""
import numpy as np
import pytest
import torch

from hftlob.config_io import builtin_config
from hftlob.data.synthetic import generate_day
from hftlob.env import MARLEnv, split_keys
from oracle import pyoracle as O

pytestmark = pytest.mark.gpu


def _float_words(env):
    L = env.layout
    fw = [L.off_world + 3, L.off_world + 4]
    for a, (k, off) in enumerate(zip(L.agent_kinds, L.agent_offsets)):
        fw += [off + 3, off + 4] if k == 0 else [off + j for j in (0, 4, 5, 6, 7, 8, 9, 10, 11, 12)]
    return np.array(fw)


def _compare_state(env, o, g, tag):
    fw = _float_words(env)
    mask = np.ones(o.shape[1], bool)
    mask[fw] = False
    bad = np.argwhere((o != g) & mask[None, :])
    assert bad.size == 0, f"{tag}: int word mismatch (env, word) {bad[:5].tolist()} oracle {o[tuple(bad[0])]} gpu {g[tuple(bad[0])]}"
    of, gf = o[:, fw].view(np.float32), g[:, fw].view(np.float32)
    assert np.allclose(of, gf, rtol=1e-5, atol=1e-5, equal_nan=True), f"{tag}: float words differ"


@pytest.mark.parametrize("name,mid", [("2_player_fq_fqc", 2_000_000), ("2_player_fq_fqc", 28_000_000),
                                      ("mm_debug_fixed_quant", 2_000_000)])
def test_env_rollout_parity(name, mid):
    cfg = builtin_config(name)
    w = cfg.world_config
    day = generate_day(n_msgs=30_000, seed=11, mid=mid, snap_every=w.n_data_msg_per_step * w.start_resolution)
    env = MARLEnv(None, cfg, data=day)
    params = env.default_params
    E, K = 64, 70                                         # crosses the 64-step episode end (auto-reset)
    init = O.init_states(env.cfg_c.lob, env.windows, day.msgs, w, env.layout.init_rec_words)
    assert (init == env._init_states.cpu().numpy()).all()
    keys = torch.from_numpy(np.arange(2 * E, dtype=np.uint32).reshape(E, 2).view(np.int32)).cuda()
    obs, state = env.reset(keys, params)
    o_state, o_obs = O.env_reset(env.cfg_c, keys.cpu().numpy().view(np.uint32), init)
    _compare_state(env, o_state, state.buf.cpu().numpy(), "reset")
    assert np.allclose(torch.cat([x.reshape(E, -1) for x in obs], 1).cpu().numpy(),
                       np.concatenate([o_obs[:, i, :d] for i, d in enumerate(
                           [env.layout.obs_dims[t] for t in env.layout.agent_types])], 1), rtol=1e-5, atol=1e-6)
    rng = keys
    for k in range(K):
        nk = split_keys(rng, 2)
        rng, sk = nk[:, 0].contiguous(), nk[:, 1].contiguous()
        acts = env.sample_actions(sk)
        o_acts = O.sample_actions(env.cfg_c, sk.cpu().numpy().view(np.uint32))
        assert (acts.cpu().numpy() == o_acts).all(), "device action sampling differs"
        prev = state.buf.cpu().numpy().copy()
        obs, state, rew, dones, info = env.step(sk, state, acts, params)
        st, oo, orw, oda, odn, oinfo = O.env_step(env.cfg_c, sk.cpu().numpy().view(np.uint32), o_acts, day.msgs,
                                                  init, prev)
        _compare_state(env, st, state.buf.cpu().numpy(), f"step {k}")
        g_rew = torch.cat([x.reshape(E, -1) for x in rew], 1).cpu().numpy()
        assert np.allclose(g_rew, orw, rtol=1e-5, atol=1e-5), f"step {k}: rewards"
        assert (dones["__all__"].cpu().numpy() == oda.astype(bool)).all()
        a0 = 0
        for t, n in enumerate(cfg.number_of_agents_per_type):
            d = env.layout.obs_dims[t]
            assert np.allclose(obs[t].cpu().numpy(), oo[:, a0:a0 + n, :d], rtol=1e-5, atol=1e-6), f"step {k}: obs type {t}"
            a0 += n
