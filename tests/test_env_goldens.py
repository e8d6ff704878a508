"""The hand-derived env-step goldens (tests/golden/env_scenarios.py) against both oracles and
the HIP env: the C oracle's full env_step, the numpy restatements (filter_messages and
ffill_best of tests/test_env_step_numpy.py, the engine scan of oracle/ref_py.py), and, with
the GPU marker, hftlob_env_step through the C ABI."""
import ctypes as C
import dataclasses
import os
import sys

import numpy as np
import pytest

from hftlob.config_io import builtin_config
from hftlob.layout import (EXE_WORDS, INFO_WORLD, INFO_WORLD_WORDS, StepOut, obs_fields, pack_env_cfg,
                           trader_ids)
from oracle import pyoracle as O
from oracle import ref_py as R
from test_env_step_numpy import ffill_best, filter_messages
from test_gpu_env import variant

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
import env_scenarios as G  # noqa: E402

I32, F32 = np.int32, np.float32
N_ROWS = 100
ABORT = [n for n, _ in INFO_WORLD].index("abort_episode")
STEP = [n for n, _ in INFO_WORLD].index("step_counter")


def golden_config():
    cfg = builtin_config("exec_debug_fixed_quants_complex")
    w = dataclasses.replace(cfg.world_config, n_data_msg_per_step=2, shuffle_action_messages=False,
                            window_selector=0, cancel_mode=1)
    cfg = dataclasses.replace(cfg, world_config=w)
    return variant(cfg, "Execution", task="sell", normalize=False, time_delay_obs_act=0, fixed_quant_value=10,
                   n_ticks_in_book=1, observation_space="engineered", action_space="fixed_quants_complex")


def _f(x):
    return np.array([x], F32).view(I32)[0]


def _side(rows, n):
    blk = np.full((n, 6), -1, I32)
    if rows:
        blk[:len(rows)] = rows
    return blk


def inputs(name):
    """(cfg, env cfg struct, layout, pre-step record [1, rec], init_states [1, init], msg_data, actions)"""
    s = G.SCENARIOS[name]
    cfg = golden_config()
    w = cfg.world_config
    assert trader_ids(cfg) == [[G.T]]
    c, L = pack_env_cfg(cfg, 1, N_ROWS, True)
    nO, nT, M, D = w.nOrders, w.nTrades, L.n_msgs, w.n_data_msg_per_step
    assert M == 10 and D == 2
    step = s.get("step", 3)
    rec = np.zeros(L.rec_words, I32)
    rec[L.off_asks:L.off_asks + 6 * nO] = _side(s["asks"], nO).ravel()
    rec[L.off_bids:L.off_bids + 6 * nO] = _side(s["bids"], nO).ravel()
    rec[L.off_trades:L.off_trades + 8 * nT] = -1
    rec[L.off_loaded:L.off_loaded + 6] = [50, 0, 0, 50, 0, step]
    rec[L.off_best_asks:L.off_best_asks + 2 * M] = np.tile(s["best_ask"], M)
    rec[L.off_best_bids:L.off_best_bids + 2 * M] = np.tile(s["best_bid"], M)
    mid = F32(F32(s["best_ask"][0] + s["best_bid"][0]) / F32(2))
    rec[L.off_world:L.off_world + 5] = [G.TIME[0], G.TIME[1], G.CNT, _f(mid), _f(0.0)]
    a = L.agent_offsets[0]
    exe = dict.fromkeys(EXE_WORDS, 0.0)
    exe.update(init_price=1000050.0, task_to_execute=600, quant_executed=0, is_sell_task=s.get("is_sell", 1),
               p_vwap=10000.5)
    for k, n in enumerate(EXE_WORDS):
        rec[a + k] = exe[n] if n in ("task_to_execute", "quant_executed", "is_sell_task") else _f(exe[n])
    init = np.zeros(L.init_rec_words, I32)
    init[L.off_asks:L.off_asks + 6 * nO] = _side(G.INIT["asks"], nO).ravel()
    init[L.off_bids:L.off_bids + 6 * nO] = _side(G.INIT["bids"], nO).ravel()
    init[L.off_trades:L.off_trades + 8 * nT] = -1
    init[L.off_loaded:L.off_loaded + 6] = G.INIT["loaded"]
    msg_data = np.array([[1, 1, 1, 100, 9000 + i, 99, 1, 0] for i in range(N_ROWS)], I32)   # unused filler
    msg_data[D * step:D * step + D] = s.get("data", G.DATA)
    acts = np.array([[s["action"]]], I32)
    return cfg, c, L, rec[None], init[None], msg_data, acts


def expected_raw(s):
    out = []
    for v in s["exp_obs_raw"]:
        out.append(F32(1) - F32(v[1]) / F32(v[2]) if isinstance(v, tuple) else v)
    return out


def check(name, L, cfg, post, obs, da, dn, info, raw, msgs):
    """One step's outputs (env 0) against the scenario's hand-derived values."""
    s = G.SCENARIOS[name]
    w = cfg.world_config
    nO, nT, M = w.nOrders, w.nTrades, L.n_msgs
    post = post[0]
    assert np.array_equal(msgs[0], np.array(s["exp_msgs"], I32)), f"{name}: combined messages"
    fields = obs_fields(cfg.dict_of_agents_configs["Execution"], w)
    want = expected_raw(s)
    for k, ((fname, dt), v) in enumerate(zip(fields, want)):
        got = raw[0, 0, k] if dt == "i" else raw[0, 0, k:k + 1].view(F32)[0]
        assert got == (v if dt == "i" else F32(v)), f"{name}: obs_raw {fname} = {got}, want {v}"
    assert bool(da[0]) == s["exp_done"], f"{name}: done"
    if not s["exp_done"]:
        assert np.array_equal(obs[0, 0, :12], np.array(want, F32)), f"{name}: obs (normalize False = raw, sorted)"
        assert np.array_equal(post[L.off_best_asks:L.off_best_asks + 2 * M].reshape(M, 2), s["exp_best_asks"])
        assert np.array_equal(post[L.off_best_bids:L.off_best_bids + 2 * M].reshape(M, 2), s["exp_best_bids"])
        assert info[0, ABORT] == s["exp_abort"], f"{name}: abort flag"
        assert np.array_equal(post[L.off_asks:L.off_asks + 6 * nO].reshape(nO, 6), _side_map(s["exp_asks"], nO))
        assert np.array_equal(post[L.off_bids:L.off_bids + 6 * nO].reshape(nO, 6), _side_map(s["exp_bids"], nO))
        tr = np.full((nT, 8), -1, I32)
        for i, r in s["exp_trades"].items():
            tr[i] = r
        assert np.array_equal(post[L.off_trades:L.off_trades + 8 * nT].reshape(nT, 8), tr), f"{name}: trades"
        wr = post[L.off_world:L.off_world + 5]
        assert (wr[0], wr[1], wr[2]) == (*s["exp_time"], s["exp_counter"])
        assert wr[3:4].view(F32)[0] == F32(s["exp_mid"])
        assert post[L.off_loaded + 5] == s["exp_step"]
        return
    # auto-reset: the record and obs are the reset's, info / obs_raw the stepped state's
    r = s["exp_reset"]
    assert np.array_equal(obs[0, 0, :12], np.array(s["exp_obs"], F32)), f"{name}: reset obs"
    assert bool(dn[0, 0]), "the stepped EXE agent is done (doom trade books the rest)"
    assert info[0, STEP] == s["exp_info_step"]
    assert np.array_equal(post[L.off_asks:L.off_asks + 6 * nO].reshape(nO, 6), _side_map(r["asks"], nO))
    assert np.array_equal(post[L.off_bids:L.off_bids + 6 * nO].reshape(nO, 6), _side_map(r["bids"], nO))
    assert (post[L.off_trades:L.off_trades + 8 * nT] == -1).all()
    assert np.array_equal(post[L.off_best_asks:L.off_best_asks + 2 * M].reshape(M, 2), [r["best_ask"]] * M)
    assert np.array_equal(post[L.off_best_bids:L.off_best_bids + 2 * M].reshape(M, 2), [r["best_bid"]] * M)
    wr = post[L.off_world:L.off_world + 5]
    assert (wr[0], wr[1], wr[2]) == (*r["time"], r["counter"])
    assert wr[3:5].view(F32).tolist() == [r["mid"], r["dt"]]
    assert post[L.off_loaded + 5] == r["step"]
    a = L.agent_offsets[0]
    e = r["exe"]
    assert post[a:a + 1].view(F32)[0] == e["init_price"] and post[a + 4:a + 5].view(F32)[0] == e["p_vwap"]
    assert (post[a + 1], post[a + 2], post[a + 3]) == (e["task"], e["executed"], e["is_sell"])
    assert not post[a + 5:a + 13].any(), "reset EXE floats are 0.0"


def _side_map(rows, n):
    blk = np.full((n, 6), -1, I32)
    for i, r in rows.items():
        blk[i] = r
    return blk


@pytest.mark.parametrize("name", list(G.SCENARIOS))
def test_c_oracle_env_step(name):
    cfg, c, L, rec, init, msg_data, acts = inputs(name)
    keys = np.zeros((1, 2), np.uint32)
    post, obs, _, da, dn, info, raw, msgs = O.env_step(c, keys, acts, msg_data, init, rec, extras=True)
    check(name, L, cfg, post, obs, da, dn, info, raw, msgs)


@pytest.mark.parametrize("name", [n for n, s in G.SCENARIOS.items() if "raw_actions" in s])
def test_numpy_restatements(name):
    """filter_messages + the order-id overwrite, the numpy engine scan and ffill_best."""
    s = G.SCENARIOS[name]
    cfg = golden_config()
    w = cfg.world_config
    act, cnl = filter_messages(np.array(s["raw_actions"], I32), np.array(s["raw_cancels"], I32))
    act[:, 4] = G.CNT - np.arange(len(act))                  # marl_env.py:285-290, zero rows included
    comb = np.concatenate([cnl, act, np.array(s.get("data", G.DATA), I32)])
    assert np.array_equal(comb, np.array(s["exp_msgs"], I32))
    ecfg = R.default_cfg(maxint=w.maxint, init_id=w.init_id, book_depth=w.book_depth, cancel_mode=w.cancel_mode,
                         type_4_interpretation=w.type_4_interpretation, check_book_fill=w.check_book_fill,
                         nOrders=w.nOrders, nTrades=w.nTrades)
    (na, nb, ntr), ba, bb = R.scan_save_bidask(ecfg, comb, _side(s["asks"], w.nOrders), _side(s["bids"], w.nOrders),
                                               np.full((w.nTrades, 8), -1, I32), (0, 0))
    assert int((ba[:, 0] == -1).any() or (bb[:, 0] == -1).any()) == s["exp_abort"]
    assert np.array_equal(ffill_best(ba, s["best_ask"][0]), s["exp_best_asks"])
    assert np.array_equal(ffill_best(bb, s["best_bid"][0]), s["exp_best_bids"])
    assert np.array_equal(na, _side_map(s["exp_asks"], w.nOrders))
    assert np.array_equal(nb, _side_map(s["exp_bids"], w.nOrders))
    for i, r in s["exp_trades"].items():
        assert np.array_equal(ntr[i], r)


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(G.SCENARIOS))
def test_hip_env_step(name):
    import torch
    from hftlob import _lib
    cfg, c, L, rec, init, msg_data, acts = inputs(name)
    dev = torch.device("cuda")
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)  # noqa: E731
    state, init_t, md, act_t = t(rec), t(init), t(msg_data), t(acts)
    keys = torch.zeros((1, 2), dtype=torch.int32, device=dev)
    A = L.obs_stride
    obs = torch.empty((1, 1, A), dtype=torch.float32, device=dev)
    rew = torch.empty((1, 1), dtype=torch.float32, device=dev)
    da = torch.empty((1,), dtype=torch.bool, device=dev)
    dn = torch.empty((1, 1), dtype=torch.bool, device=dev)
    info = torch.empty((1, L.info_words), dtype=torch.int32, device=dev)
    raw = torch.empty((1, 1, A), dtype=torch.int32, device=dev)
    msgs = torch.empty((1, L.n_msgs, 8), dtype=torch.int32, device=dev)
    out = StepOut(*[_lib.ptr(x) for x in (obs, rew, da, dn, info, raw, msgs)])
    _lib.check(_lib.lib().hftlob_env_step(C.byref(c), 1, _lib.ptr(keys), _lib.ptr(act_t), _lib.ptr(md),
                                          _lib.ptr(init_t), _lib.ptr(state), C.byref(out),
                                          _lib.stream_ptr(device=dev)))
    torch.cuda.synchronize()
    n = lambda x: x.cpu().numpy()  # noqa: E731
    check(name, L, cfg, n(state), n(obs), n(da), n(dn), n(info), n(raw), n(msgs))
