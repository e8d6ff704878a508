"""The hand-derived market-maker goldens of the metric config (tests/golden/mm_scenarios.py)
against the C oracle's env_step, the numpy restatements (fixed_quant_rows of
tests/test_mm_actions.py, getCancelMsgs / _filter_messages / _ffill_best_prices of
tests/test_env_step_numpy.py, the numpy engine of oracle/ref_py.py, the numpy MM reward with
the unwind trade, mm_obs_numpy) and, with the GPU marker, hftlob_env_step through the C ABI.

Float expectations are evaluated here in float32, in the reference expression's order
(mm_env.py:2414-2430, 2642; weak-typed Python constants stay f32): every term of these
scenarios is exact in float32, so the oracle and the HIP env must match them to the last bit
(asserted with rtol 1e-6)."""
import ctypes as C
import dataclasses
import os
import sys

import numpy as np
import pytest

from hftlob.config_io import builtin_config
from hftlob.layout import EXE_WORDS, INFO_MM, INFO_WORLD, INFO_WORLD_WORDS, StepOut, pack_env_cfg, trader_ids
from oracle import pyoracle as O
from oracle import ref_py as R
from test_env_step_numpy import cancel_msgs, ffill_best, filter_messages
from test_exe_variants import expected_rows as exe_rows
from test_gpu_env import variant
from test_mm_actions import fixed_quant_rows, mm_obs_numpy

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
import mm_scenarios as G  # noqa: E402

I32, F = np.int32, np.float32
N_ROWS = 100
ABORT = [n for n, _ in INFO_WORLD].index("abort_episode")
STEP = [n for n, _ in INFO_WORLD].index("step_counter")
MMI = {n: k for k, (n, _) in enumerate(INFO_MM)}
P, Q, PT, AT = 0, 1, 6, 7


def mm_golden_config():
    cfg = builtin_config("2_player_fq_fqc")
    w = dataclasses.replace(cfg.world_config, n_data_msg_per_step=2, shuffle_action_messages=False,
                            window_selector=0)
    return variant(dataclasses.replace(cfg, world_config=w), "Execution", task="sell")


def _fb(x):
    return np.array([x], F).view(I32)[0]


def _side(rows, n):
    blk = np.full((n, 6), -1, I32)
    if rows:
        blk[:len(rows)] = rows
    return blk


def _side_map(rows, n):
    blk = np.full((n, 6), -1, I32)
    for i, r in rows.items():
        blk[i] = r
    return blk


def inputs(name):
    """(cfg, env cfg struct, layout, pre-step record [1, rec], init_states [1, init], msg_data, actions [1, 2])"""
    s = G.SCENARIOS[name]
    cfg = mm_golden_config()
    w = cfg.world_config
    assert trader_ids(cfg) == [[G.T], [G.TE]]
    c, L = pack_env_cfg(cfg, 1, N_ROWS, True)
    nO, nT, M, D = w.nOrders, w.nTrades, L.n_msgs, w.n_data_msg_per_step
    assert M == 14 and D == 2 and L.agent_kinds == [0, 1]
    step = s.get("step", 3)
    rec = np.zeros(L.rec_words, I32)
    rec[L.off_asks:L.off_asks + 6 * nO] = _side(s["asks"], nO).ravel()
    rec[L.off_bids:L.off_bids + 6 * nO] = _side(s["bids"], nO).ravel()
    rec[L.off_trades:L.off_trades + 8 * nT] = -1
    rec[L.off_loaded:L.off_loaded + 6] = [50, 0, 0, 50, 0, step]
    rec[L.off_best_asks:L.off_best_asks + 2 * M] = np.tile(s["best_ask"], M)
    rec[L.off_best_bids:L.off_best_bids + 2 * M] = np.tile(s["best_bid"], M)
    mid = F(F(s["best_ask"][0] + s["best_bid"][0]) / F(2))
    rec[L.off_world:L.off_world + 5] = [G.TIME[0], G.TIME[1], G.CNT, _fb(mid), _fb(0.0)]
    a = L.agent_offsets[0]
    mm = s["mm"]
    rec[a:a + 5] = [0, 0, mm["inv"], _fb(mm["total"]), _fb(mm["cash"])]
    x = L.agent_offsets[1]
    exe = dict.fromkeys(EXE_WORDS, 0.0)
    exe.update(init_price=1000150.0, task_to_execute=600, quant_executed=0, is_sell_task=1, p_vwap=10001.5)
    for k, n in enumerate(EXE_WORDS):
        rec[x + k] = exe[n] if n in ("task_to_execute", "quant_executed", "is_sell_task") else _fb(exe[n])
    init = np.zeros(L.init_rec_words, I32)
    init[L.off_asks:L.off_asks + 6 * nO] = _side(G.INIT["asks"], nO).ravel()
    init[L.off_bids:L.off_bids + 6 * nO] = _side(G.INIT["bids"], nO).ravel()
    init[L.off_trades:L.off_trades + 8 * nT] = -1
    init[L.off_loaded:L.off_loaded + 6] = G.INIT["loaded"]
    msg_data = np.array([[1, 1, 1, 100, 9000 + i, 99, 1, 0] for i in range(N_ROWS)], I32)   # unused filler
    msg_data[D * step:D * step + D] = s["data"]
    acts = np.array([[s["action"], 0]], I32)
    return cfg, c, L, rec[None], init[None], msg_data, acts


def expected_reward(s):
    """reward_spooner_asym_damped2 (mm_env.py:2430) in float32, in the reference's order."""
    r = s["exp_reward"]
    cfg = mm_golden_config().dict_of_agents_configs["MarketMaking"]
    reb = F(F(r["rebate_value"]) * F(cfg.rebate_bps / 10_000))
    inv_pnl = F(F(F(r["inv"]) * F(F(r["mid_end"]) - F(r["mid_old"]))) / F(100))
    damp = F(F(cfg.inventoryPnL_gamma) * F(inv_pnl - F(max(F(0), F(F(cfg.inventoryPnL_eta) * inv_pnl)))))
    reward = F(F(F(F(r["buy"]) + F(r["sell"])) + reb) + damp)
    return reward, F(reward / F(cfg.reward_scaling_quo)), inv_pnl


def _close(got, want, what):
    assert np.isclose(F(got), F(want), rtol=1e-6, atol=1e-7), f"{what}: got {got!r}, want {want!r}"


def check(name, L, cfg, post, obs, rew, da, info, msgs):
    """One step's outputs (env 0) against the scenario's hand-derived values."""
    s = G.SCENARIOS[name]
    w = cfg.world_config
    nO, nT, M = w.nOrders, w.nTrades, L.n_msgs
    post = post[0]
    assert np.array_equal(msgs[0], np.array(s["exp_msgs"], I32)), f"{name}: combined messages"
    reward, scaled, inv_pnl = expected_reward(s)
    fi = info[0].view(F)
    base = INFO_WORLD_WORDS
    _close(fi[base + MMI["reward"]], reward, f"{name}: info reward")
    _close(fi[base + MMI["reward_spooner_asym_damped2"]], reward, f"{name}: info reward_spooner_asym_damped2")
    _close(rew[0, 0], scaled, f"{name}: reward / reward_scaling_quo")
    _close(fi[base + MMI["invPnL"]], inv_pnl, f"{name}: InventoryPnL")
    _close(fi[base + MMI["buyPnL"]], s["exp_reward"]["buy"], f"{name}: buyPnL")
    _close(fi[base + MMI["sellPnL"]], s["exp_reward"]["sell"], f"{name}: sellPnL")
    for k, v in s["exp_info"].items():
        assert info[0, base + MMI[k]] == v, f"{name}: info {k} = {info[0, base + MMI[k]]}, want {v}"
    want_obs = np.array([F(F(v) / F(d)) for v, d in s["exp_obs"]], F)
    assert np.array_equal(obs[0, 0, :2], want_obs), f"{name}: MM basic obs {obs[0, 0, :2]} want {want_obs}"
    assert bool(da[0]) == s["exp_done"], f"{name}: done"
    if s["exp_done"]:
        assert info[0, STEP] == s["exp_info_step"]
        a = L.agent_offsets[0]
        assert np.array_equal(post[a:a + 5], np.zeros(5, I32)), "the reset MM state is all zeros"
        assert np.array_equal(post[L.off_asks:L.off_asks + 6 * nO].reshape(nO, 6), _side(G.INIT["asks"], nO))
        assert np.array_equal(post[L.off_bids:L.off_bids + 6 * nO].reshape(nO, 6), _side(G.INIT["bids"], nO))
        return
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
    assert wr[3:4].view(F)[0] == F(s["exp_mid"])
    assert post[L.off_loaded + 5] == s["exp_step"]
    a = L.agent_offsets[0]
    m, pre = s["exp_mm_state"], s["mm"]
    assert (post[a], post[a + 1], post[a + 2]) == (m["bid_dist"], m["ask_dist"], m["inv"]), f"{name}: MM state"
    _close(post[a + 3:a + 4].view(F)[0], F(F(pre["total"]) + F(m["pnl"])), f"{name}: total_PnL")
    _close(post[a + 4:a + 5].view(F)[0], F(F(pre["cash"]) + F(m["pnl"])), f"{name}: cash_balance")


@pytest.mark.parametrize("name", list(G.SCENARIOS))
def test_c_oracle_mm_goldens(name):
    cfg, c, L, rec, init, msg_data, acts = inputs(name)
    keys = np.zeros((1, 2), np.uint32)
    post, obs, rew, da, dn, info, raw, msgs = O.env_step(c, keys, acts, msg_data, init, rec, extras=True)
    check(name, L, cfg, post, obs, rew, da, info, msgs)


def mm_reward_with_unwind(t, w, tr, ba, bb, inv, old_mid, tid, ep_done):
    """get_reward (mm_env.py:2247-2430) in float64 from the step's trades and forward-filled best
    quotes, with the fictional unwind trade of an episode's last step (:2285-2317)."""
    tick = w.tick_size
    tr = tr.astype(np.int64).copy()

    def split(trades):
        ex = np.where((trades[:, P] >= 0)[:, None], trades, 0)
        mine = (tid == ex[:, PT]) | (tid == ex[:, AT])
        ag = np.where(mine[:, None], ex, 0)
        buy = ((ag[:, Q] >= 0) & (tid == ag[:, PT])) | ((ag[:, Q] < 0) & (tid == ag[:, AT]))
        sel = ((ag[:, Q] < 0) & (tid == ag[:, PT])) | ((ag[:, Q] >= 0) & (tid == ag[:, AT]))
        pb = (ag[:, Q] >= 0) & (tid == ag[:, PT])
        ps = (ag[:, Q] < 0) & (tid == ag[:, PT])
        return tuple(np.where(m[:, None], ag, 0) for m in (buy, sel, pb, ps))

    B, S_, _, _ = split(tr)
    inv_b = inv + np.abs(B[:, Q]).sum() - np.abs(S_[:, Q]).sum()
    last_mid = (bb[-1] + ba[-1]) / 2
    unwind_row = None
    if ep_done and inv_b != 0:
        assert t.unwind_price == "mid"
        pen = t.unwind_price_penalty * tick * (1 if inv_b > 0 else -1)
        row = [int(last_mid - pen), np.sign(inv_b) * abs(inv_b), w.artificial_order_id_end_episode,
               w.placeholder_order_id, 0, 0, w.artificial_trader_id_end_episode, tid]
        unwind_row = int(np.nonzero((tr == -1).any(1))[0][0])    # add_trade: first row holding any -1
        tr[unwind_row] = row
    B, S_, PB, PS = split(tr)
    ref = last_mid
    buy_pnl = ((ref - B[:, P]) / tick * np.abs(B[:, Q])).sum()
    sell_pnl = ((S_[:, P] - ref) / tick * np.abs(S_[:, Q])).sum()
    rebate_value = (PB[:, P] / tick * np.abs(PB[:, Q])).sum() + (PS[:, P] / tick * np.abs(PS[:, Q])).sum()
    inv_pnl = inv * (last_mid - old_mid) / tick
    new_inv = inv + np.abs(B[:, Q]).sum() - np.abs(S_[:, Q]).sum()
    income = (S_[:, P] / tick * np.abs(S_[:, Q])).sum()
    outgoing = (B[:, P] / tick * np.abs(B[:, Q])).sum()
    return dict(buy=buy_pnl, sell=sell_pnl, rebate_value=rebate_value, inv_pnl=inv_pnl, new_inv=new_inv,
                forced_unwind=inv_b * ep_done, unwind_row=unwind_row, unwind=None if unwind_row is None
                else tr[unwind_row].tolist(), income=income, outgoing=outgoing, mid_end=last_mid)


@pytest.mark.parametrize("name", list(G.SCENARIOS))
def test_numpy_restatements_mm_goldens(name):
    """the action rows (fixed_quant_rows), getCancelMsgs + _filter_messages + order ids, the numpy
    engine scan, _ffill_best_prices, the MM reward with the unwind trade and the basic obs"""
    s = G.SCENARIOS[name]
    cfg, c, L, rec, init, msg_data, acts = inputs(name)
    rec = rec[0]
    w = cfg.world_config
    tm, te = cfg.dict_of_agents_configs["MarketMaking"], cfg.dict_of_agents_configs["Execution"]
    nO, M = w.nOrders, L.n_msgs
    mm_rows = fixed_quant_rows(tm, w, rec, L, G.T, s["action"])
    assert mm_rows == s["exp_mm_rows"]
    t0, t1 = G.TIME
    asks, bids = _side(s["asks"], nO), _side(s["bids"], nO)
    act = np.array([[ty, sd, q, p, w.placeholder_order_id, G.T, t0, t1] for ty, sd, q, p in mm_rows], I32)
    cnl = np.concatenate([cancel_msgs(bids, G.T, 1, 1, t0, t1), cancel_msgs(asks, G.T, 1, -1, t0, t1)])
    act, cnl = filter_messages(act, cnl)
    e_rows = np.array([[1, -1, q, p, w.placeholder_order_id, G.TE, t0, t1]
                       for q, p in exe_rows(te, w, rec, L, L.agent_offsets[1], 0)], I32)
    e_cnl = cancel_msgs(asks, G.TE, 4, -1, t0, t1)
    e_rows, e_cnl = filter_messages(e_rows, e_cnl)
    actions = np.concatenate([act, e_rows])
    actions[:, 4] = G.CNT - np.arange(len(actions))                   # marl_env.py:285-290
    comb = np.concatenate([cnl, e_cnl, actions, np.array(s["data"], I32)])
    assert np.array_equal(comb, np.array(s["exp_msgs"], I32)), "combined messages"
    ecfg = R.default_cfg(maxint=w.maxint, init_id=w.init_id, book_depth=w.book_depth, cancel_mode=w.cancel_mode,
                         type_4_interpretation=w.type_4_interpretation, check_book_fill=w.check_book_fill,
                         nOrders=w.nOrders, nTrades=w.nTrades)
    (na, nb, ntr), ba, bb = R.scan_save_bidask(ecfg, comb, asks, bids, np.full((w.nTrades, 8), -1, I32), (0, 0))
    assert int((ba[:, 0] == -1).any() or (bb[:, 0] == -1).any()) == s["exp_abort"]
    fba, fbb = ffill_best(ba, s["best_ask"][0]), ffill_best(bb, s["best_bid"][0])
    assert np.array_equal(fba, s["exp_best_asks"]) and np.array_equal(fbb, s["exp_best_bids"])
    tr = np.full((w.nTrades, 8), -1, I32)
    for i, r in s["exp_trades"].items():
        tr[i] = r
    assert np.array_equal(ntr, tr), "trades"
    if not s["exp_done"]:
        assert np.array_equal(na, _side_map(s["exp_asks"], nO)) and np.array_equal(nb, _side_map(s["exp_bids"], nO))
    mm = s["mm"]
    old_mid = float(rec[L.off_world + 3:L.off_world + 4].view(F)[0])
    got = mm_reward_with_unwind(tm, w, ntr, fba[:, 0].astype(np.float64), fbb[:, 0].astype(np.float64), mm["inv"],
                                old_mid, G.T, s["exp_done"])
    r = s["exp_reward"]
    assert (got["buy"], got["sell"], got["rebate_value"]) == (r["buy"], r["sell"], r["rebate_value"])
    assert got["mid_end"] == r["mid_end"] and old_mid == r["mid_old"]
    assert got["new_inv"] == s["exp_info"]["inventory"] and got["forced_unwind"] == s["exp_info"]["forced_unwind"]
    if s["exp_done"]:
        assert got["unwind_row"] == s["exp_unwind_row"] and got["unwind"] == s["exp_unwind"]
        assert (got["income"], got["outgoing"]) == (s["exp_pnl_terms"]["income"], s["exp_pnl_terms"]["outgoing"])
        return
    assert got["income"] - got["outgoing"] == s["exp_mm_state"]["pnl"]
    # the basic observation from the stepped record (mm_obs_numpy reads the post-step words)
    post = rec.copy()
    post[L.off_best_asks:L.off_best_asks + 2 * M] = fba.ravel()
    post[L.off_best_bids:L.off_best_bids + 2 * M] = fbb.ravel()
    post[L.agent_offsets[0] + 2] = got["new_inv"]
    want = [F(F(v) / F(d)) for v, d in s["exp_obs"]]
    assert mm_obs_numpy(tm, w, post, L, L.agent_offsets[0]) == want


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(G.SCENARIOS))
def test_hip_mm_goldens(name):
    import torch
    from hftlob import _lib
    cfg, c, L, rec, init, msg_data, acts = inputs(name)
    dev = torch.device("cuda")
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)  # noqa: E731
    state, init_t, md, act_t = t(rec), t(init), t(msg_data), t(acts)
    keys = torch.zeros((1, 2), dtype=torch.int32, device=dev)
    A = L.obs_stride
    obs = torch.empty((1, 2, A), dtype=torch.float32, device=dev)
    rew = torch.empty((1, 2), dtype=torch.float32, device=dev)
    da = torch.empty((1,), dtype=torch.bool, device=dev)
    dn = torch.empty((1, 2), dtype=torch.bool, device=dev)
    info = torch.empty((1, L.info_words), dtype=torch.int32, device=dev)
    msgs = torch.empty((1, L.n_msgs, 8), dtype=torch.int32, device=dev)
    out = StepOut(*[_lib.ptr(x) for x in (obs, rew, da, dn, info)], None, _lib.ptr(msgs))
    _lib.check(_lib.lib().hftlob_env_step(C.byref(c), 1, _lib.ptr(keys), _lib.ptr(act_t), _lib.ptr(md),
                                          _lib.ptr(init_t), _lib.ptr(state), C.byref(out),
                                          _lib.stream_ptr(device=dev)))
    torch.cuda.synchronize()
    n = lambda x: x.cpu().numpy()  # noqa: E731
    check(name, L, cfg, n(state), n(obs), n(rew), n(da), n(info), n(msgs))
