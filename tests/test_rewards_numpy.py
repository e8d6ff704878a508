"""Rewards of the C oracle against a numpy restatement written from the reference
lines: MM get_reward (mm_env.py:2247-2673, with _extract_agent_trade_stats :2214-2243)
and EXE get_reward (exec_env.py:1511-1758, get_agent_trades JaxOrderBookArrays.py:895-904),
on env states reached by oracle rollouts.  The numpy side computes in float64 from the
step's trades and (forward-filled) best quotes, so floats are compared with a tolerance
of 1e-5 of the magnitude of the terms that form them (f32 rounding, summation order).
Steps that end an episode are skipped: their trades are replaced by the auto-reset."""

import numpy as np
import pytest

from hftlob.config_io import builtin_config
from hftlob.data.synthetic import generate_day
from hftlob.data.windows import make_windows
from hftlob.layout import INFO_AGENT_WORDS, INFO_EXE, INFO_MM, INFO_WORLD_WORDS, pack_env_cfg, trader_ids
from oracle import pyoracle as O
from test_gpu_env import variant

P, Q, PT, AT = 0, 1, 6, 7          # TradesFeat columns (jaxob_constants)


def _f(rec, i):
    return float(rec[i:i + 1].view(np.float32)[0])


def _close(a, b, scale, what):
    assert abs(a - b) <= 1e-5 * max(1.0, abs(b), scale), f"{what}: oracle {a} numpy {b} (scale {scale})"


def mm_reward_numpy(t, w, prev, post, L, a_off, tid):
    """mm_env.py:2247-2440 for a step that does not end the episode (no fictional unwind trade)."""
    tick, M = w.tick_size, L.n_msgs
    tr = post[L.off_trades:L.off_trades + 8 * w.nTrades].reshape(-1, 8).astype(np.int64)
    ex = np.where((tr[:, P] >= 0)[:, None], tr, 0)
    mine = (tid == ex[:, PT]) | (tid == ex[:, AT])
    ag = np.where(mine[:, None], ex, 0)
    other = np.where(mine[:, None], 0, ex)
    buy = ((ag[:, Q] >= 0) & (tid == ag[:, PT])) | ((ag[:, Q] < 0) & (tid == ag[:, AT]))
    sel = ((ag[:, Q] < 0) & (tid == ag[:, PT])) | ((ag[:, Q] >= 0) & (tid == ag[:, AT]))
    pbuy = (ag[:, Q] >= 0) & (tid == ag[:, PT])
    psel = (ag[:, Q] < 0) & (tid == ag[:, PT])
    B, S_ = np.where(buy[:, None], ag, 0), np.where(sel[:, None], ag, 0)
    PB, PS = np.where(pbuy[:, None], ag, 0), np.where(psel[:, None], ag, 0)
    ba = post[L.off_best_asks:L.off_best_asks + 2 * M].reshape(M, 2)[:, 0].astype(np.float64)
    bb = post[L.off_best_bids:L.off_best_bids + 2 * M].reshape(M, 2)[:, 0].astype(np.float64)
    avg_mid = ((bb + ba) / 2).mean()
    last_mid = (bb[-1] + ba[-1]) / 2
    st = prev[a_off:a_off + 5]
    inv, cash = int(st[2]), _f(prev, a_off + 4)
    income = (S_[:, P] / tick * np.abs(S_[:, Q])).sum()
    outgoing = (B[:, P] / tick * np.abs(B[:, Q])).sum()
    bq, sq = np.abs(B[:, Q]).sum(), np.abs(S_[:, Q]).sum()
    new_inv = inv + bq - sq
    rebate = ((PB[:, P] / tick * np.abs(PB[:, Q])).sum() + (PS[:, P] / tick * np.abs(PS[:, Q])).sum()) * (
        t.rebate_bps / 10_000)
    rp = t.reference_price
    if rp == "mid_avg":
        ref_buy = ref_sell = ref = avg_mid
    elif rp == "mid":
        ref_buy = ref_sell = ref = last_mid
    elif rp == "far_touch":
        ref_buy, ref_sell = ba[-1], bb[-1]
        ref = ref_buy if new_inv > 0 else ref_sell
    else:
        ref_buy, ref_sell = bb[-1], ba[-1]
        ref = ref_buy if new_inv > 0 else ref_sell
    pnl = income - outgoing + rebate
    new_cash = cash + pnl
    inv_value = new_inv * ref / tick
    other_q = np.abs(other[:, Q]).sum()
    traded = bq + sq
    market_share = traded / (traded + other_q) if traded + other_q else float("nan")
    old_mid = _f(prev, L.off_world + 3)
    inv_pnl = inv * (last_mid - old_mid) / tick
    buy_pnl = ((ref_buy - B[:, P]) / tick * np.abs(B[:, Q])).sum()
    sell_pnl = ((S_[:, P] - ref_sell) / tick * np.abs(S_[:, Q])).sum()
    eta, gamma = t.inventoryPnL_eta, t.inventoryPnL_gamma
    out = {
        "reward_spooner": buy_pnl + sell_pnl + rebate + inv_pnl,
        "reward_spooner_damped": buy_pnl + sell_pnl + rebate + inv_pnl - eta * inv_pnl,
        "reward_spooner_asym_damped": buy_pnl + sell_pnl + rebate + inv_pnl - max(0.0, eta * inv_pnl),
        "reward_spooner_asym_damped2": buy_pnl + sell_pnl + rebate + gamma * (inv_pnl - max(0.0, eta * inv_pnl)),
        "reward_portfolio_value": new_inv * (ref / tick) + new_cash,
        "buyPnL": buy_pnl, "sellPnL": sell_pnl, "invPnL": inv_pnl, "inventoryValue": inv_value,
        "delta_mid_price": last_mid - old_mid, "market_share": market_share,
    }
    if rp in ("mid", "mid_avg"):
        old_ref = old_mid
    else:
        oba = prev[L.off_best_asks + 2 * (M - 1)]
        obb = prev[L.off_best_bids + 2 * (M - 1)]
        old_ref = (oba if inv > 0 else obb) if rp == "far_touch" else (obb if inv > 0 else oba)
    out["reward_delta_pv"] = (new_cash + inv_value) - (old_ref / tick * inv + cash)
    scale = income + outgoing + abs(inv_pnl) + abs(new_inv * ref / tick) + abs(new_cash) + abs(buy_pnl) + abs(sell_pnl)
    return out, new_inv, scale


def exe_reward_numpy(t, w, prev, post, L, a_off, tid):
    """exec_env.py:1511-1731 for a step that does not end the episode (no doom trade)."""
    tick, M = w.tick_size, L.n_msgs
    tr = post[L.off_trades:L.off_trades + 8 * w.nTrades].reshape(-1, 8).astype(np.int64)
    ex = np.where((tr[:, P] >= 0)[:, None], tr, 0)
    mine = (tid == ex[:, PT]) | (tid == ex[:, AT])
    ag = np.where(mine[:, None], ex, 0)
    other = np.where(mine[:, None], 0, ex)
    st = prev[a_off:a_off + 13]
    init_price, task, qe, sell = _f(prev, a_off), int(st[1]), int(st[2]), int(st[3])
    ba = post[L.off_best_asks:L.off_best_asks + 2 * M].reshape(M, 2)[:, 0].astype(np.float64)
    bb = post[L.off_best_bids:L.off_best_bids + 2 * M].reshape(M, 2)[:, 0].astype(np.float64)
    avg_mid = ((bb + ba) / 2).mean()
    aq, oq = int(np.abs(ag[:, Q]).sum()), int(np.abs(other[:, Q]).sum())
    if oq == 0:
        p_vwap = avg_mid // tick
    else:
        p_vwap = ((other[:, P] // tick) * (np.abs(other[:, Q]) / oq)).sum()
    qp = int(((ag[:, P] // tick) * np.abs(ag[:, Q])).sum())
    d = 1 if sell else -1
    adv = d * (qp - p_vwap * aq)
    drift = d * aq * (p_vwap - init_price // tick)
    out = {"advantage": adv, "drift": drift, "reward_normal": adv + t.reward_lambda * drift,
           "quant_left": task - qe - aq}
    slip = np.where(mine, ag[:, P] - init_price, 0.0)          # rows of other traders weigh |q| = 0
    out["reward_simplest_case"] = float(((slip if sell else -slip) * np.abs(ag[:, Q])).sum())
    scale = abs(qp) + abs(p_vwap * aq) + abs(aq * init_price / tick) + np.abs(ag[:, P] * ag[:, Q]).sum()
    return out, scale


CASES = [dict(), dict(mm=dict(reference_price="far_touch")), dict(mm=dict(reference_price="mid_avg")),
         dict(mm=dict(reference_price="near_touch", reward_function="spooner")),
         dict(exe=dict(reference_price="mid", task="buy")), dict(exe=dict(reward_function="simplest_case")),
         dict(exe=dict(reward_function="simplest_case", task="buy"))]


@pytest.mark.parametrize("case", CASES, ids=lambda d: ",".join(f"{k}:{v}" for k, v in d.items()) or "metric")
def test_rewards_vs_numpy(case):
    cfg = builtin_config("2_player_fq_fqc")
    if "mm" in case:
        cfg = variant(cfg, "MarketMaking", **case["mm"])
    if "exe" in case:
        cfg = variant(cfg, "Execution", **case["exe"])
    w = cfg.world_config
    day = generate_day(n_msgs=20_000, seed=8, snap_every=w.n_data_msg_per_step * w.start_resolution)
    win = make_windows(day, w)
    c, L = pack_env_cfg(cfg, len(win.starts), day.msgs.shape[0], True)
    init = O.init_states(c.lob, win, day.msgs, w, L.init_rec_words)
    tm, te = cfg.dict_of_agents_configs["MarketMaking"], cfg.dict_of_agents_configs["Execution"]
    (tid_mm,), (tid_exe,) = trader_ids(cfg)
    E = 16
    keys = np.arange(2 * E, dtype=np.uint32).reshape(E, 2) + 3
    st, _ = O.env_reset(c, keys, init)
    checked = traded = 0
    for k in range(40):
        acts = O.sample_actions(c, keys + 7 * k)
        post, _, rew, done_all, _, info = O.env_step(c, keys + 7 * k, acts, day.msgs, init, st)
        fi = info.view(np.float32)
        for e in range(E):
            if done_all[e]:
                continue
            mm, new_inv, s_mm = mm_reward_numpy(tm, w, st[e], post[e], L, L.agent_offsets[0], tid_mm)
            base = INFO_WORLD_WORDS
            for name, v in mm.items():
                j = [n for n, _ in INFO_MM].index(name)
                got = float(fi[e, base + j])
                if name == "market_share" and np.isnan(v):
                    assert np.isnan(got)
                    continue
                _close(got, v, s_mm, f"step {k} env {e} MM {name}")
            assert info[e, base + [n for n, _ in INFO_MM].index("inventory")] == new_inv
            key = {"delta_portfolio_value": "reward_delta_pv"}.get(tm.reward_function, "reward_" + tm.reward_function)
            _close(float(fi[e, base]), mm[key], s_mm, "MM reward")
            ex, s_ex = exe_reward_numpy(te, w, st[e], post[e], L, L.agent_offsets[1], tid_exe)
            base = INFO_WORLD_WORDS + INFO_AGENT_WORDS
            names = [n for n, _ in INFO_EXE]
            _close(float(fi[e, base + names.index("advantage")]), ex["advantage"], s_ex, "EXE advantage")
            _close(float(fi[e, base + names.index("drift")]), ex["drift"], s_ex, "EXE drift")
            _close(float(fi[e, base + names.index("reward")]), ex["reward_normal"], s_ex, "EXE info reward")
            assert info[e, base + names.index("quant_left")] == ex["quant_left"]
            want = ex["reward_simplest_case"] if te.reward_function == "simplest_case" else ex["reward_normal"]
            _close(float(rew[e, 1]) * te.reward_scaling_quo, want, s_ex, "EXE reward")
            checked += 1
            traded += s_ex > 0
        st = post
    assert checked > 400 and traded > 20
