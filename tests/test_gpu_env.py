"""Fused env step parity: HIP hftlob_env_step vs the CPU oracle over episodes.

Integer words of the state record (book, trades, best arrays, ids, counters)
must be bit-exact; float words, obs and rewards within rtol = atol = 1e-5.
"""
import dataclasses

import numpy as np
import pytest
import torch

from hftlob.config_io import builtin_config
from hftlob.data.synthetic import generate_day
from hftlob.env import MARLEnv, split_keys
from oracle import pyoracle as O

pytestmark = pytest.mark.gpu

RTOL = ATOL = 1e-5


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
    assert np.allclose(of, gf, rtol=RTOL, atol=RTOL, equal_nan=True), f"{tag}: float words differ"


def _compare_info(env, o, g, tag):
    from hftlob.layout import AGENT_MM, INFO_AGENT_WORDS, INFO_EXE, INFO_MM, INFO_WORLD, INFO_WORLD_WORDS
    isf = np.zeros(o.shape[1], bool)
    for k, (_, f) in enumerate(INFO_WORLD):
        isf[k] = f
    for a, kind in enumerate(env.layout.agent_kinds):
        for k, (_, f) in enumerate(INFO_MM if kind == AGENT_MM else INFO_EXE):
            isf[INFO_WORLD_WORDS + a * INFO_AGENT_WORDS + k] = f
    bad = np.argwhere((o != g) & ~isf[None, :])
    assert bad.size == 0, f"{tag}: info int word mismatch {bad[:5].tolist()}"
    assert np.allclose(o[:, isf].view(np.float32), g[:, isf].view(np.float32), rtol=RTOL, atol=ATOL,
                       equal_nan=True), f"{tag}: info float words differ"


def _compare_obs_raw(env, t, a0, n, g, o_raw, o_msgs, tag):
    """info["agents"][t]["obs_raw"] vs the oracle's raw words: int32 fields bit-exact, float32 fields
    within RTOL; the messages space: the step's messages, bit-exact."""
    fields = env.obs_raw_fields[t]
    if fields is None:
        assert np.array_equal(g.cpu().numpy(), np.broadcast_to(o_msgs[:, None], g.shape)), f"{tag}: raw messages"
        return
    assert list(g) == [f for f, _ in fields]
    for k, (name, dt) in enumerate(fields):
        col = o_raw[:, a0:a0 + n, k]
        got = g[name].cpu().numpy()
        if dt == "i":
            assert got.dtype == np.int32 and np.array_equal(got, col), f"{tag}: obs_raw {name}"
        else:
            assert got.dtype == np.float32 and np.allclose(got, col.view(np.float32), rtol=RTOL, atol=ATOL), \
                f"{tag}: obs_raw {name}"


def variant(cfg, type_name, **changes):
    """A copy of `cfg` with fields of one agent type replaced (configs are frozen dataclasses)."""
    agents = dict(cfg.dict_of_agents_configs)
    agents[type_name] = dataclasses.replace(agents[type_name], **changes)
    return dataclasses.replace(cfg, dict_of_agents_configs=agents)


_DAYS = {}


def _day(w, mid, seed=11):
    key = (mid, seed, w.n_data_msg_per_step * w.start_resolution)
    if key not in _DAYS:
        _DAYS[key] = generate_day(n_msgs=30_000, seed=seed, mid=mid, snap_every=key[2])
    return _DAYS[key]


def rollout_parity(cfg, mid=2_000_000, E=64, K=70, seed=11, partitionable=True, day=None):
    w = cfg.world_config
    day = _day(w, mid, seed) if day is None else day
    env = MARLEnv(None, cfg, data=day, prng_partitionable=partitionable)
    params = env.default_params
    init = O.init_states(env.cfg_c.lob, env.windows, day.msgs, w, env.layout.init_rec_words)
    assert (init == env._init_states.cpu().numpy()).all()
    keys = torch.from_numpy(np.arange(2 * E, dtype=np.uint32).reshape(E, 2).view(np.int32)).cuda()
    obs, state = env.reset(keys, params)
    o_state, o_obs = O.env_reset(env.cfg_c, keys.cpu().numpy().view(np.uint32), init)
    _compare_state(env, o_state, state.buf.cpu().numpy(), "reset")
    msg_t = env.message_obs_types
    for t in range(len(obs)):
        if msg_t[t]:
            assert obs[t].dtype == torch.int32 and not obs[t].any(), "messages reset obs is blank"
    assert np.allclose(torch.cat([x.reshape(E, -1) for t, x in enumerate(obs) if not msg_t[t]], 1).cpu().numpy(),
                       np.concatenate([o_obs[:, i, :env.layout.obs_dims[t]] for i, t in enumerate(
                           env.layout.agent_types) if not msg_t[t]], 1), rtol=RTOL, atol=1e-6)
    extras = env.save_raw_observations or any(msg_t)
    rng = keys
    for k in range(K):
        nk = split_keys(rng, 2, partitionable)
        rng, sk = nk[:, 0].contiguous(), nk[:, 1].contiguous()
        acts = env.sample_actions(sk)
        o_acts = O.sample_actions(env.cfg_c, sk.cpu().numpy().view(np.uint32))
        assert (acts.cpu().numpy() == o_acts).all(), "device action sampling differs"
        prev = state.buf.cpu().numpy().copy()
        obs, state, rew, dones, info = env.step(sk, state, acts, params)
        res = O.env_step(env.cfg_c, sk.cpu().numpy().view(np.uint32), o_acts, day.msgs, init, prev, extras=extras)
        st, oo, orw, oda, odn, oinfo = res[:6]
        _compare_state(env, st, state.buf.cpu().numpy(), f"step {k}")
        g_rew = torch.cat([x.reshape(E, -1) for x in rew], 1).cpu().numpy()
        assert np.allclose(g_rew, orw, rtol=RTOL, atol=ATOL), f"step {k}: rewards"
        assert (dones["__all__"].cpu().numpy() == oda.astype(bool)).all()
        a0 = 0
        for t, n in enumerate(cfg.number_of_agents_per_type):
            d = env.layout.obs_dims[t]
            g_dn = dones["agents"][t].cpu().numpy()
            assert (g_dn == odn[:, a0:a0 + n].astype(bool)).all(), f"step {k}: dones type {t}"
            if msg_t[t]:  # the step's messages, blank where the agent is done or the env resets
                zero = (odn[:, a0:a0 + n].astype(bool) | oda.astype(bool)[:, None])[:, :, None, None]
                want = np.where(zero, 0, res[7][:, None])
                assert np.array_equal(obs[t].cpu().numpy(), want), f"step {k}: messages obs type {t}"
            else:
                assert np.allclose(obs[t].cpu().numpy(), oo[:, a0:a0 + n, :d], rtol=RTOL, atol=1e-6), \
                    f"step {k}: obs type {t}"
            if env.save_raw_observations:
                _compare_obs_raw(env, t, a0, n, info["agents"][t]["obs_raw"], res[6], res[7], f"step {k}")
            a0 += n
        _compare_info(env, oinfo, env.last_info_words.cpu().numpy(), f"step {k}")


def _raw(cfg):
    return dataclasses.replace(cfg, world_config=dataclasses.replace(cfg.world_config, save_raw_observations=True))


@pytest.mark.parametrize("mm,exe", [("basic", "engineered"), ("engineered", "basic"), ("engineered", "simplest_case"),
                                    ("messages", "engineered")])
def test_save_raw_observations_parity(mm, exe):
    """info["agents"][t]["obs_raw"] under save_raw_observations (marl_env.py:684-685), the MM
    "messages" observation (mm_env.py:2820-2821), normalised and not."""
    cfg = _raw(builtin_config("2_player_fq_fqc"))
    for norm in (True, False):
        c = variant(variant(cfg, "MarketMaking", observation_space=mm, normalize=norm), "Execution",
                    observation_space=exe, normalize=norm)
        rollout_parity(c, E=32, K=40 if norm else 12)


def test_save_raw_observations_fixed_time(tmp_path_factory):
    day = _loaded("fixed_time", str(tmp_path_factory.mktemp("lob")))
    cfg = builtin_config("2_player_fq_fqc")
    w = dataclasses.replace(cfg.world_config, ep_type="fixed_time", episode_time=300, start_resolution=300,
                            save_raw_observations=True)
    cfg = variant(dataclasses.replace(cfg, world_config=w), "MarketMaking", observation_space="engineered")
    rollout_parity(cfg, E=16, K=20, day=day)


def test_messages_obs_multi_agent_rollout():
    """Two MM agents on the messages space, then the sampled rollout (per_step outputs) with
    save_raw_observations: every step's raw records == an oracle replay from the same keys."""
    cfg = variant(builtin_config("2_player_fq_fqc"), "MarketMaking", observation_space="messages")
    cfg = dataclasses.replace(cfg, number_of_agents_per_type=[2, 1])
    rollout_parity(cfg, E=16, K=20)
    cfg = _raw(variant(cfg, "Execution", observation_space="basic"))
    env = MARLEnv(None, cfg, data=_day(cfg.world_config, 2_000_000))
    params = env.default_params
    E, T, M = 16, 6, env.layout.n_msgs
    keys = torch.from_numpy(np.arange(2 * E, dtype=np.uint32).reshape(E, 2).view(np.int32)).cuda()
    _, state = env.reset(keys, params)
    st = state.buf.cpu().numpy()
    k_in = torch.tensor([0, 7], dtype=torch.int32, device="cuda")
    k_out = torch.empty_like(k_in)
    obs, _, _, dones, info = env.rollout_sampled(k_in, k_out, state, params, T, per_step=True, n_slices=1)
    assert obs[0].shape == (T, E, 2, M, 8) and obs[0].dtype == torch.int32
    raw_m = info["agents"][0]["obs_raw"].reshape(T, E, 2, M, 8).cpu().numpy()
    raw_e = {k: v.reshape(T, E, 1).cpu().numpy() for k, v in info["agents"][1]["obs_raw"].items()}
    assert list(raw_e) == ["best_ask_price", "best_bid_price", "remaining_quant"]
    init = env._init_states.cpu().numpy()
    rng = k_in.reshape(1, 2)
    for k in range(T):
        ks = split_keys(rng, E + 1, True)[0]
        rng, sk = ks[0:1].contiguous(), ks[1:].contiguous()
        sk_np = sk.cpu().numpy().view(np.uint32)
        acts = O.sample_actions(env.cfg_c, sk_np)
        st, _, _, oda, odn, _, oraw, omsgs = O.env_step(env.cfg_c, sk_np, acts, env.data.msgs, init, st, extras=True)
        assert np.array_equal(raw_m[k], np.broadcast_to(omsgs[:, None], (E, 2, M, 8))), f"step {k}: raw msgs"
        for j, name in enumerate(raw_e):
            assert np.array_equal(raw_e[name][k], oraw[:, 2:3, j]), f"step {k}: {name}"
        zero = (odn[:, :2].astype(bool) | oda.astype(bool)[:, None])[:, :, None, None]
        assert np.array_equal(obs[0][k].cpu().numpy(), np.where(zero, 0, omsgs[:, None])), f"step {k}: obs"


@pytest.mark.parametrize("name,mid", [("2_player_fq_fqc", 2_000_000), ("2_player_fq_fqc", 28_000_000),
                                      ("mm_debug_fixed_quant", 2_000_000),
                                      ("3_player_fq_fqc_dir", 2_000_000),
                                      ("exec_debug_fixed_quants_complex", 2_000_000)])
def test_env_rollout_parity(name, mid):
    rollout_parity(builtin_config(name), mid)


_LOADED = {}


def _loaded(ep_type, tmp_root):
    """A generated raw LOBSTER day through hftlob.data.lobster (LoadLOBSTER_resample)."""
    from hftlob.data import lobster as Lb
    from hftlob.data.raw_synthetic import write_raw_lobster_day
    if "root" not in _LOADED:
        write_raw_lobster_day(tmp_root, n_events=30_000, seed=5, mid=2_000_000)
        _LOADED["root"] = tmp_root
    root = _LOADED["root"]
    if ep_type == "fixed_steps":
        ld = Lb.LoadLOBSTER_resample(root, root, 10, "fixed_steps", window_length=64, window_resolution=16,
                                     n_data_msg_per_step=100, stock="SYN", time_period="2026_Oct")
        return Lb.LoadedDay.from_arrays(*ld.run_loading("gpu_fs"))
    ld = Lb.LoadLOBSTER_resample(root, root, 10, "fixed_time", window_length=300, window_resolution=300,
                                 n_data_msg_per_step=100, stock="SYN", time_period="2026_Oct")
    return Lb.LoadedDay.from_arrays(*ld.run_loading("gpu_ft"))


@pytest.mark.parametrize("nT", [100, 8])
def test_env_trade_rows_neg1_fields(nT):
    """Replayed executions (type 4) with order id -1 or time -1: the step's trade log takes its next
    row at the first col 4 (TIME) == -1 (JaxOrderBookArrays.py:205), so trades of time -1 messages
    are overwritten and those of oid -1 messages kept; nT = 8 also overflows the log every step."""
    cfg = builtin_config("2_player_fq_fqc")
    cfg = dataclasses.replace(cfg, world_config=dataclasses.replace(cfg.world_config, nTrades=nT))
    base = _day(cfg.world_config, 2_000_000)
    msgs = base.msgs.copy()
    rng = np.random.Generator(np.random.PCG64(7))
    u = rng.random(len(msgs))
    ex = msgs[:, 0] == 4
    msgs[:, 4] = np.where(ex & (u < 0.3), -1, msgs[:, 4])
    msgs[:, 6] = np.where(ex & (u >= 0.3) & (u < 0.6), -1, msgs[:, 6])
    day = dataclasses.replace(base, msgs=msgs)
    rollout_parity(cfg, E=32, K=66, day=day)


@pytest.mark.parametrize("ep_type", ["fixed_steps", "fixed_time"])
def test_env_rollout_parity_lobster_loaded(ep_type, tmp_path_factory):
    """Raw LOBSTER files -> loader -> env: fixed_steps windows, and fixed_time windows with the
    data-row time mask (base_env.py:358-367) and the 15-field EXE obs (exec_env.py:1940-2010)."""
    day = _loaded(ep_type, str(tmp_path_factory.mktemp("lob")))
    cfg = builtin_config("2_player_fq_fqc")
    w = dataclasses.replace(cfg.world_config, ep_type=ep_type,
                            episode_time=64 if ep_type == "fixed_steps" else 300,
                            start_resolution=16 if ep_type == "fixed_steps" else 300)
    cfg = dataclasses.replace(cfg, world_config=w)
    rollout_parity(cfg, E=32, K=40, day=day)
    for norm in (False,):
        rollout_parity(variant(cfg, "Execution", normalize=norm), E=16, K=12, day=day)


@pytest.mark.parametrize("mode,part", [(2, True), (3, True), (3, False)])
def test_env_rollout_parity_random_cancel(mode, part):
    """cancel_mode 2/3: the engine's random cancel fallback draws from the step's scan key."""
    cfg = builtin_config("2_player_fq_fqc")
    cfg = dataclasses.replace(cfg, world_config=dataclasses.replace(cfg.world_config, cancel_mode=mode))
    rollout_parity(cfg, E=32, K=66, partitionable=part)


@pytest.mark.parametrize("name", ["2_player_fq_fqc", "3_player_fq_fqc_dir"])
def test_env_rollout_parity_legacy_prng(name):
    """jax_threefry_partitionable=False (the pre-0.5 JAX default) split / random_bits."""
    rollout_parity(builtin_config(name), E=32, K=66, partitionable=False)


MM_VARIANTS = [
    dict(reward_function=r) for r in ("portfolio_value", "buy_sell_pnl", "complex", "zero_inv", "spooner",
                                      "spooner_damped", "spooner_asym_damped", "spooner_scaled",
                                      "delta_portfolio_value")
] + [
    dict(reference_price="mid_avg", unwind_price="mid_avg"),
    dict(reference_price="far_touch", unwind_price="far_touch"),
    dict(reference_price="near_touch", inv_penalty="linear"),
    dict(inv_penalty="quadratic", clip_reward=True),
    dict(inv_penalty="exp4", inv_penalty_lambda=1e-6),
    dict(inv_penalty="threshold", exclude_extreme_spreads=True, volume_traded_bonus="market_share"),
    dict(auto_liquidate_threshold=3, normalize=False),
]


@pytest.mark.parametrize("changes", MM_VARIANTS, ids=lambda d: ",".join(f"{k}={v}" for k, v in d.items()))
def test_mm_option_parity(changes):
    rollout_parity(variant(builtin_config("2_player_fq_fqc"), "MarketMaking", **changes), E=32, K=66)


MM_ACTION_VARIANTS = [
    dict(action_space="bobRL", bob_v0=1), dict(action_space="bobRL", bob_v0=2, fixed_quant_value=3),
    dict(action_space="bobRL", bob_v0=5), dict(action_space="bobRL", bob_v0=10),
    dict(action_space="bobStrategy", bob_v0=2), dict(action_space="bobStrategy", bob_v0=5, fixed_quant_value=1),
    dict(action_space="AvSt"), dict(action_space="AvSt", avst_k_parameter=1.5, avst_var_parameter=2000.0),
    dict(action_space="spread_skew"),
    dict(action_space="spread_skew", multiplier_type="spread", spread_multiplier=2.0, skew_multiplier=0.5),
    dict(action_space="simple"), dict(action_space="simple", simple_nothing_action=False, n_ticks_offset=2),
    dict(action_space="simple", sell_buy_all_option=True, fixed_quant_value=2),
    dict(action_space="bobRL", bob_v0=2, fixed_action_setting=True, fixed_action=3),
    dict(action_space="fixed_quants", sell_buy_all_option=True),            # 9-entry tables (mm_env.py:1018-1023)
    dict(action_space="fixed_quants", sell_buy_all_option=True, fixed_quant_value=2, tenth_action="NA"),
    dict(action_space="bobRL", bob_v0=2, sell_buy_all_option=True),          # the flag is not read by bobRL
]


@pytest.mark.parametrize("changes", MM_ACTION_VARIANTS, ids=lambda d: ",".join(f"{k}={v}" for k, v in d.items()))
def test_mm_action_space_parity(changes):
    """MM action spaces bobRL / bobStrategy / AvSt / spread_skew / simple (mm_env.py:1123-1809)."""
    rollout_parity(variant(builtin_config("2_player_fq_fqc"), "MarketMaking", **changes), E=32, K=66)


def test_mm_avst_fixed_time(tmp_path_factory):
    """AvSt's time_left under fixed_time episodes (mm_env.py:1287-1290) on loader-built windows."""
    day = _loaded("fixed_time", str(tmp_path_factory.mktemp("lob")))
    cfg = builtin_config("2_player_fq_fqc")
    w = dataclasses.replace(cfg.world_config, ep_type="fixed_time", episode_time=300, start_resolution=300)
    cfg = variant(dataclasses.replace(cfg, world_config=w), "MarketMaking", action_space="AvSt",
                  avst_var_parameter=500.0)
    rollout_parity(cfg, E=32, K=20, day=day)


@pytest.mark.parametrize("norm", [True, False])
def test_mm_engineered_fixed_time(norm, tmp_path_factory):
    """MM engineered obs under fixed_time episodes: 10 sorted keys incl. delta_time and
    time_remaining (mm_env.py:3029-3088, observation_space :3195-3198)."""
    day = _loaded("fixed_time", str(tmp_path_factory.mktemp("lob")))
    cfg = builtin_config("2_player_fq_fqc")
    w = dataclasses.replace(cfg.world_config, ep_type="fixed_time", episode_time=300, start_resolution=300)
    cfg = variant(dataclasses.replace(cfg, world_config=w), "MarketMaking", observation_space="engineered",
                  normalize=norm)
    rollout_parity(cfg, E=32, K=20, day=day)


EXE_VARIANTS = [dict(reward_function="finish_fast"), dict(reference_price="mid", task="buy"),
                dict(reward_function="simplest_case"), dict(reward_function="simplest_case", task="buy"),
                dict(task="sell", normalize=False),
                dict(doom_price_penalty=0.1),                    # Python-float penalty: f32 far-touch price
                dict(doom_price_penalty=0.37, reference_price="mid"),
                dict(action_space="simplest_case"), dict(action_space="simplest_case", task_size=25),
                dict(action_space="fixed_quants_1msg"), dict(action_space="fixed_quants_1msg", task_size=40),
                dict(action_space="twap"), dict(action_space="twap", task_size=7, task="buy"),
                dict(observation_space="basic"), dict(observation_space="basic", normalize=False),
                dict(observation_space="simplest_case"), dict(observation_space="simplest_case", normalize=False),
                # fixed_prices: MultiDiscrete([fixed_quant_value] * n_actions) quantities per price level
                dict(action_space="fixed_prices", n_actions=4, fixed_quant_value=11),
                dict(action_space="fixed_prices", n_actions=4, fixed_quant_value=11, task_size=30, task="sell"),
                dict(action_space="fixed_prices", n_actions=3, fixed_quant_value=11, task="buy"),
                dict(action_space="fixed_prices", n_actions=2, fixed_quant_value=11, task_size=12),
                dict(action_space="fixed_prices", n_actions=1, fixed_quant_value=10)]


@pytest.mark.parametrize("changes", EXE_VARIANTS, ids=lambda d: ",".join(f"{k}={v}" for k, v in d.items()))
def test_exe_option_parity(changes):
    rollout_parity(variant(builtin_config("2_player_fq_fqc"), "Execution", **changes), E=32, K=66)


@pytest.mark.parametrize("name,part,exe", [("2_player_fq_fqc", True, None), ("3_player_fq_fqc_dir", True, None),
                                           ("2_player_fq_fqc", False, None), ("2_player_fq_fqc", True, 3),
                                           ("exec_debug_fixed_quants_complex", False, 2)])
def test_step_sampled_equals_split_sample_step(name, part, exe):
    """hftlob_env_step_sampled (one launch) == split_keys + sample_actions + env_step
    (exe = n: the Execution type uses fixed_prices with n MultiDiscrete quantities)."""
    cfg = builtin_config(name)
    if exe:
        cfg = variant(cfg, "Execution", action_space="fixed_prices", n_actions=exe, fixed_quant_value=11)
    w = cfg.world_config
    env = MARLEnv(None, cfg, data=_day(w, 2_000_000), prng_partitionable=part)
    params = env.default_params
    E = 48
    keys = torch.from_numpy(np.arange(2 * E, dtype=np.uint32).reshape(E, 2).view(np.int32)).cuda()
    _, s1 = env.reset(keys, params)
    s2 = s1.clone(env)
    kbuf = [torch.tensor([0, 7], dtype=torch.int32, device="cuda"), torch.empty(2, dtype=torch.int32, device="cuda")]
    rng = kbuf[0].clone().reshape(1, 2)
    acts_out = torch.empty((E, env.action_words), dtype=torch.int32, device="cuda")
    for k in range(70):
        o1, s1, r1, d1, _ = env.step_sampled(kbuf[k % 2], kbuf[(k + 1) % 2], s1, params, acts_out)
        o1 = [x.clone() for x in o1]
        r1 = [x.clone() for x in r1]
        da1 = d1["__all__"].clone()
        ks = split_keys(rng, E + 1, part)[0]
        rng, sk = ks[0:1].contiguous(), ks[1:].contiguous()
        acts = env.sample_actions(sk)
        o2, s2, r2, d2, _ = env.step(sk, s2, acts, params)
        assert (acts_out == acts).all(), f"step {k}: sampled actions"
        assert (kbuf[(k + 1) % 2] == rng[0]).all(), f"step {k}: carried key"
        assert (s1.buf == s2.buf).all(), f"step {k}: state"
        assert all((a == b).all() for a, b in zip(o1, o2)) and all((a == b).all() for a, b in zip(r1, r2))
        assert (da1 == d2["__all__"]).all()


def _named_config(name):
    """builtin configs, or "speed_A_B": Speed_test's MultiAgentConfig() with [A, B] agents and 100
    data messages (32-step episodes, speed_test_config)"""
    if name.startswith("speed_"):
        a, b = (int(x) for x in name.split("_")[1:])
        return speed_test_config([a, b], 100)
    return builtin_config(name)


@pytest.mark.parametrize("name,part,exe,T,per_step,G", [("2_player_fq_fqc", True, None, 70, False, 0),
                                                          ("speed_5_5", True, None, 70, False, 0),
                                                          ("speed_5_5", True, None, 7, True, 0),
                                                          ("speed_5_5", False, None, 9, True, 0),
                                                          ("speed_10_10", True, None, 70, False, 0),
                                                          ("speed_10_10", True, None, 7, True, 0),
                                                          ("2_player_fq_fqc", True, None, 7, True, 0),
                                                          ("3_player_fq_fqc_dir", False, None, 13, True, 0),
                                                          ("exec_debug_fixed_quants_complex", False, 2, 9, True, 0),
                                                          ("2_player_fq_fqc", True, None, 70, False, 4),
                                                          ("2_player_fq_fqc", True, None, 7, True, 3),
                                                          ("2_player_fq_fqc", True, None, 5, True, 1),
                                                          ("3_player_fq_fqc_dir", False, None, 13, True, 2),
                                                          ("exec_debug_fixed_quants_complex", False, 2, 9, True, 4)])
def test_rollout_sampled_equals_step_sampled(name, part, exe, T, per_step, G):
    """hftlob_env_rollout_sampled (T steps over G env slices on their own streams; G = 0: one
    k_env_rollout launch, every env's T steps back to back) == T
    hftlob_env_step_sampled launches: state, carried key, and (per_step) every step's
    actions / obs / rewards / dones, bit for bit; the rollout crosses an auto-reset."""
    cfg = _named_config(name)
    if exe:
        cfg = variant(cfg, "Execution", action_space="fixed_prices", n_actions=exe, fixed_quant_value=11)
    w = cfg.world_config
    env = MARLEnv(None, cfg, data=_day(w, 2_000_000), prng_partitionable=part)
    if name.startswith("speed_"):  # the rows-alias instantiation (k_env_rollout<2, 100, false, true>)
        assert env.launch_info()["rows_alias"] == 1
    params = env.default_params
    E = 40
    keys = torch.from_numpy(np.arange(2 * E, dtype=np.uint32).reshape(E, 2).view(np.int32)).cuda()
    _, s1 = env.reset(keys, params)
    s2 = s1.clone(env)
    k0 = torch.tensor([3, 9], dtype=torch.int32, device="cuda")
    # prefix of steps so the T-step launch crosses the episode end
    pre = 60 if T < 70 else 0
    kbuf = [k0.clone(), torch.empty(2, dtype=torch.int32, device="cuda")]
    for k in range(pre):
        env.step_sampled(kbuf[k % 2], kbuf[(k + 1) % 2], s1, params)
    s2 = s1.clone(env)
    kin = kbuf[pre % 2].clone()
    ref_acts, ref_obs, ref_rew, ref_done = [], [], [], []
    acts_out = torch.empty((E, env.action_words), dtype=torch.int32, device="cuda")
    for k in range(pre, pre + T):
        o1, s1, r1, d1, _ = env.step_sampled(kbuf[k % 2], kbuf[(k + 1) % 2], s1, params, acts_out)
        ref_acts.append(acts_out.clone())
        ref_obs.append([x.clone() for x in o1])
        ref_rew.append([x.clone() for x in r1])
        ref_done.append(d1["__all__"].clone())
    kout = torch.empty(2, dtype=torch.int32, device="cuda")
    shape = (T, E, env.action_words) if per_step else (E, env.action_words)
    acts2 = torch.empty(shape, dtype=torch.int32, device="cuda")
    o2, s2, r2, d2, _ = env.rollout_sampled(kin, kout, s2, params, T, per_step=per_step, actions_out=acts2,
                                            n_slices=G)
    assert (kout == kbuf[(pre + T) % 2]).all(), "carried key"
    assert (s1.buf == s2.buf).all(), "state after the rollout"
    steps = range(T) if per_step else [T - 1]
    for t in steps:
        pick = (lambda x: x[t]) if per_step else (lambda x: x)  # noqa: E731
        assert (pick(acts2) == ref_acts[t]).all(), f"step {t}: actions"
        assert all((pick(a) == b).all() for a, b in zip(o2, ref_obs[t])), f"step {t}: obs"
        assert all((pick(a) == b).all() for a, b in zip(r2, ref_rew[t])), f"step {t}: rewards"
        assert (pick(d2["__all__"]) == ref_done[t]).all(), f"step {t}: done"


def test_rollout_sampled_graph_capture():
    """a 2-slice rollout_sampled captured in a HIP graph (the slice stream joins the capture through
    the fork / join events) replays to the same state and carried key as the eager call"""
    cfg = builtin_config("2_player_fq_fqc")
    env = MARLEnv(None, cfg, data=_day(cfg.world_config, 2_000_000), persistent_outputs=True)
    params = env.default_params
    E, T = 64, 10
    keys = torch.from_numpy(np.arange(2 * E, dtype=np.uint32).reshape(E, 2).view(np.int32)).cuda()
    _, s1 = env.reset(keys, params)
    s2 = s1.clone(env)
    s_start = s1.clone(env)
    k0 = torch.tensor([4, 2], dtype=torch.int32, device="cuda")
    kin, kout = k0.clone(), torch.empty(2, dtype=torch.int32, device="cuda")
    env.rollout_sampled(kin, kout, s1, params, T, n_slices=2)
    torch.cuda.synchronize()
    gin, gout = torch.empty(2, dtype=torch.int32, device="cuda"), torch.empty(2, dtype=torch.int32, device="cuda")
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):                      # warm-up outside the capture (library streams, events)
        gin.copy_(k0)
        env.rollout_sampled(gin, gout, s2, params, T, n_slices=2)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        env.rollout_sampled(gin, gout, s2, params, T, n_slices=2)
    s2.buf.copy_(s_start.buf)
    gin.copy_(k0)
    g.replay()
    torch.cuda.synchronize()
    assert (gout == kout).all() and (s2.buf == s1.buf).all()


def test_rollout_sampled_random_cancel():
    """the cancel_mode 2/3 instantiation of the multi-step kernel: a 66-step launch == 66 launches"""
    cfg = builtin_config("2_player_fq_fqc")
    cfg = dataclasses.replace(cfg, world_config=dataclasses.replace(cfg.world_config, cancel_mode=3))
    env = MARLEnv(None, cfg, data=_day(cfg.world_config, 2_000_000))
    params = env.default_params
    E = 24
    keys = torch.from_numpy(np.arange(2 * E, dtype=np.uint32).reshape(E, 2).view(np.int32)).cuda()
    _, s1 = env.reset(keys, params)
    s2 = s1.clone(env)
    kbuf = [torch.tensor([1, 2], dtype=torch.int32, device="cuda"), torch.empty(2, dtype=torch.int32, device="cuda")]
    kin = kbuf[0].clone()
    for k in range(66):
        env.step_sampled(kbuf[k % 2], kbuf[(k + 1) % 2], s1, params)
    kout = torch.empty(2, dtype=torch.int32, device="cuda")
    env.rollout_sampled(kin, kout, s2, params, 66, n_slices=3)
    assert (kout == kbuf[0]).all() and (s1.buf == s2.buf).all()


@pytest.mark.parametrize("name,agents,changes", [
    ("2_player_fq_fqc", [3, 2], None),                     # several agents of each type
    ("3_player_fq_fqc_dir", [2, 2, 3], None),
    ("2_player_fq_fqc", [2, 3], dict(action_space="fixed_prices", n_actions=3, fixed_quant_value=11)),
    ("mm_debug_fixed_quant", [4], None),
])
def test_multi_agent_per_type_parity(name, agents, changes):
    """number_of_agents_per_type > 1: trader ids, per-agent key splits, the action / cancel row
    layout and the shuffle over more rows (marl_env.py:85-115,254-315)."""
    cfg = builtin_config(name)
    if changes:
        cfg = variant(cfg, "Execution", **changes)
    cfg = dataclasses.replace(cfg, number_of_agents_per_type=agents)
    rollout_parity(cfg, E=24, K=66)


def test_max_book_size_parity():
    """nOrders = nTrades = HFTLOB_MAX_SLOTS (256): four slot sets per lane in the env kernel."""
    cfg = builtin_config("2_player_fq_fqc")
    cfg = dataclasses.replace(cfg, world_config=dataclasses.replace(cfg.world_config, nOrders=256, nTrades=256))
    rollout_parity(cfg, E=16, K=40)


SWEEP = [(ag, D) for ag in ([1, 1], [5, 5], [10, 10]) for D in (100, 1)]


def speed_test_config(agents, D, episode_time=32):
    """Speed_test.py:50-71, 101-113: MultiAgentConfig() (MM bobRL + EXE fixed_quants_complex) with
    agents per type and n_data_msg_per_step D; the parity runs use 32-step episodes (the bench
    rows keep the default 6400) so a short rollout crosses the auto-reset."""
    cfg = builtin_config("default")
    w = dataclasses.replace(cfg.world_config, n_data_msg_per_step=D, episode_time=episode_time,
                            start_resolution=episode_time)
    return dataclasses.replace(cfg, world_config=w, number_of_agents_per_type=list(agents))


@pytest.mark.parametrize("agents,D", SWEEP, ids=lambda x: str(x))
def test_speed_test_sweep_parity(agents, D):
    """Speed_test's sweep ([1,1] / [5,5] / [10,10] agents x 100 / 1 data messages; [10,10] is 120
    agent message rows): env.step vs the oracle over an auto-reset, then the sampled rollout
    (the bench path, 2 slices) vs the oracle's C rollout loop: state and carried key."""
    cfg = speed_test_config(agents, D)
    rollout_parity(cfg, E=16, K=40)
    env = MARLEnv(None, cfg, data=_day(cfg.world_config, 2_000_000))
    params = env.default_params
    E, T = 24, 40
    keys = torch.from_numpy(np.arange(2 * E, dtype=np.uint32).reshape(E, 2).view(np.int32) + 5).cuda()
    _, state = env.reset(keys, params)
    s0 = state.buf.cpu().numpy()
    k_in = torch.tensor([0, 42], dtype=torch.int32, device="cuda")
    k_out = torch.empty_like(k_in)
    env.rollout_sampled(k_in, k_out, state, params, T, n_slices=2)
    o_st, o_key = O.rollout_sampled(env.cfg_c, k_in.cpu().numpy().view(np.uint32), env.data.msgs,
                                    env._init_states.cpu().numpy(), s0, T)
    _compare_state(env, o_st, state.buf.cpu().numpy(), "rollout_sampled")
    assert (k_out.cpu().numpy().view(np.uint32) == o_key).all(), "carried key"


@pytest.mark.parametrize("agents,D,E", [([5, 5], 100, 24), ([5, 5], 1, 24), ([5, 5], 100, 4000), ([5, 5], 1, 4000),
                                        ([10, 10], 100, 24), ([10, 10], 1, 24), ([10, 10], 100, 4000),
                                        ([10, 10], 1, 4000)], ids=lambda x: str(x))
def test_speed_test_rows_alias_persistent(agents, D, E):
    """Speed_test's [5, 5] and [10, 10] agents at their default launch: ONE persistent k_env_rollout
    launch of the rows-alias instantiation (k_env_rollout<2, 100, false, true>: the 60 / 120 agent
    message rows live inside the trade log, [10, 10]'s over two message chunks whose second is read
    into registers with the first, trades_fill after that, the book resident in LDS from step to step),
    at 24 envs and at the sweep's 4000 envs, 70 steps over 32-step episodes so every env crosses
    two auto-resets; end state and carried master key against the oracle's C rollout loop
    (Speed_test.py:50-71,186-196).  hftlob_env_launch_info asserts the instantiation."""
    cfg = speed_test_config(agents, D)
    env = MARLEnv(None, cfg, data=_day(cfg.world_config, 2_000_000), return_info=False, persistent_outputs=True)
    info = env.launch_info()
    assert (info["nfix"], info["rows_alias"], info["random_cancel"]) == (100, 1, 0)
    assert info["lds_bytes"] == env.lds_bytes_per_env() and info["lds_bytes"] * 16 <= env.LDS_PER_CU
    assert env.default_slices(E) == 0, "the default launch is the persistent one"
    params = env.default_params
    T = 70
    keys = split_keys(torch.zeros((1, 2), dtype=torch.int32, device="cuda"), E + 1)[0]
    _, state = env.reset(keys[1:].contiguous(), params)
    s0 = state.buf.cpu().numpy()
    kin, kout = keys[0].clone(), torch.empty(2, dtype=torch.int32, device="cuda")
    env.rollout_sampled(kin, kout, state, params, T)  # n_slices = default_slices(E) = 0
    torch.cuda.synchronize()
    o_st, o_key = O.rollout_sampled(env.cfg_c, kin.cpu().numpy().view(np.uint32), env.data.msgs,
                                    env._init_states.cpu().numpy(), s0, T)
    _compare_state(env, o_st, state.buf.cpu().numpy(), f"{agents} x {D} persistent rollout, {E} envs")
    assert (kout.cpu().numpy().view(np.uint32) == o_key).all(), "carried key"
    assert (state.world_state.step_counter.cpu().numpy() < T).all(), "every env crossed its episode end"


def _ref_configs():
    import json
    import os
    p = os.path.join(os.path.dirname(__file__), "golden", "reference_env_configs.json")
    with open(p) as f:
        return json.load(f)


@pytest.mark.parametrize("fname", sorted(_ref_configs()))
def test_reference_env_config_runs(fname):
    """Every env config the reference ships (config/env_configs/*.json, serialised into
    tests/golden/reference_env_configs.json by tests/golden/make_reference_env_configs.py) runs on
    the HIP env and matches the oracle over 24 steps."""
    from hftlob.config_io import dict_to_multiagent_config
    cfg = dict_to_multiagent_config(_ref_configs()[fname])
    rollout_parity(cfg, E=16, K=24)


def test_concurrent_persistent_rollouts():
    """Two persistent rollouts on two streams at once (their waves share SIMDs and the kernel's
    issue-priority table, k_env_rollout's balance_prio), and a batch larger than the GPU holds at
    once (later workgroups reuse the hardware wave slots of finished ones): each equals the same
    rollout run alone, bit for bit.  The priority rule orders issue, never results."""
    cfg = builtin_config("2_player_fq_fqc")
    env = MARLEnv(None, cfg, data=_day(cfg.world_config, 2_000_000))
    params = env.default_params
    T = 70  # crosses the auto-reset
    runs = []
    for E, seed in ((3000, 1), (2000, 2), (9000, 3)):
        keys = torch.from_numpy((np.arange(2 * E, dtype=np.uint32).reshape(E, 2) + 7 * seed).view(np.int32)).cuda()
        _, s = env.reset(keys, params)
        runs.append((E, s, torch.tensor([seed, 5], dtype=torch.int32, device="cuda")))
    ref = []
    for E, s, k0 in runs:  # alone
        s1 = s.clone(env)
        kout = torch.empty(2, dtype=torch.int32, device="cuda")
        env.rollout_sampled(k0.clone(), kout, s1, params, T, n_slices=0)
        torch.cuda.synchronize()
        ref.append((s1.buf.clone(), kout.clone()))
    streams = [torch.cuda.Stream() for _ in runs[:2]]
    outs = []
    for (E, s, k0), st in zip(runs[:2], streams):  # the first two concurrently
        st.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(st):
            s2 = s.clone(env)
            kout = torch.empty(2, dtype=torch.int32, device="cuda")
            env.rollout_sampled(k0.clone(), kout, s2, params, T, n_slices=0)
            outs.append((s2, kout))
    torch.cuda.synchronize()
    for (s2, kout), (rs, rk) in zip(outs, ref[:2]):
        assert (s2.buf == rs).all() and (kout == rk).all()
    # the over-full batch, again alone: the same as its first run (no dependence on slot reuse)
    E, s, k0 = runs[2]
    s3 = s.clone(env)
    kout = torch.empty(2, dtype=torch.int32, device="cuda")
    env.rollout_sampled(k0.clone(), kout, s3, params, T, n_slices=0)
    torch.cuda.synchronize()
    assert (s3.buf == ref[2][0]).all() and (kout == ref[2][1]).all()
