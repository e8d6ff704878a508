"""MM action spaces: the C oracle's action messages vs a numpy restatement written from
mm_env.py (bobRL :1474-1561, bobStrategy :1400-1472, AvSt :1248-1398, spread_skew
:1667-1808, simple :1123-1246), on env states reached by oracle rollouts.  float32
arithmetic follows the jnp expressions (weak-typed Python scalars stay f32).
"""
import math

import numpy as np
import pytest

from hftlob.config_io import builtin_config
from hftlob.data.synthetic import generate_day
from hftlob.data.windows import make_windows
from hftlob.layout import pack_env_cfg
from oracle import pyoracle as O
from test_gpu_env import variant

F = np.float32


def _fdiv(a, b):
    """jnp.floor_divide on float32 (x - fmod) / y, corrected toward -inf."""
    a, b = F(a), F(b)
    m = F(math.fmod(a, b))
    d = F((a - m) / b)
    if m != 0 and ((b < 0) != (m < 0)):
        d = F(d - F(1))
    return F(round(float(d)))


def _cvt(x):
    return int(np.clip(np.float64(x), -2**31, 2**31 - 1)) if np.isfinite(x) else 0


def _gather(a, n):
    i = a + n if a < 0 else a
    return min(max(i, 0), n - 1)


def _masked_best(asks, bids, tid, maxint):
    pa = np.where(asks[:, 3] != tid, asks[:, 0], -1)
    pb = np.where(bids[:, 3] != tid, bids[:, 0], -1)
    mn = np.where(pa == -1, maxint, pa).min()
    return (-1 if mn == maxint else int(mn)), int(pb.max())


def expected(cfg_t, w, rec, L, tid, action, inv):
    """(bid_quant, ask_quant, bid_price, ask_price) of the two action rows."""
    tick, maxint = w.tick_size, w.maxint
    nO = w.nOrders
    asks = rec[L.off_asks:L.off_asks + 6 * nO].reshape(nO, 6)
    bids = rec[L.off_bids:L.off_bids + 6 * nO].reshape(nO, 6)
    M = L.n_msgs
    lba, lbb = int(rec[L.off_best_asks + (M - 1) * 2]), int(rec[L.off_best_bids + (M - 1) * 2])
    if cfg_t.fixed_action_setting:
        action = cfg_t.fixed_action
    a = cfg_t.action_space
    fq = cfg_t.fixed_quant_value
    if a in ("bobRL", "bobStrategy", "AvSt"):
        ba, bb = _masked_best(asks, bids, tid, maxint)
        empty = ba == -1 or bb == -1
        ba, bb = (ba // tick) * tick, (bb // tick) * tick
        if empty:
            ba, bb = lba, lbb
        if a == "bobRL":
            tabs = {1: ([1, 2, 0], [1, 0, 2]), 2: ([2, 3, 1, 4, 0], [2, 1, 3, 0, 4]),
                    5: ([5, 6, 4, 7, 3, 8, 2, 9, 1, 10, 0], [5, 4, 6, 3, 7, 2, 8, 1, 9, 0, 10]),
                    10: ([10, 11, 9, 12, 8, 13, 7, 14, 6, 15, 5, 16, 4, 17, 3, 18, 2, 19, 1, 20, 0],
                         [10, 9, 11, 8, 12, 7, 13, 6, 14, 5, 15, 4, 16, 3, 17, 2, 18, 1, 19, 0, 20])}
            tb, ta = tabs[cfg_t.bob_v0]
            i = _gather(action, len(tb))
            bq, aq = (0, 0) if empty else (tb[i] * fq, ta[i] * fq)
            return bq, aq, bb, ba
        if a == "bobStrategy":
            kappa = F(action + 1) / F(cfg_t.bob_v0 * 5)
            v0 = F(cfg_t.bob_v0)
            bq = int(np.rint(v0 * max(F(1) - kappa * F(inv), F(0))))
            aq = int(np.rint(v0 * max(F(1) + kappa * F(inv), F(0))))
            return (0, 0, bb, ba) if empty else (bq, aq, bb, ba)
        mid = (ba + bb) // 2
        gamma = F([0.1, 0.2, 0.5, 1, 2, 5, 10, 20][_gather(action, 8)])
        k = F(cfg_t.avst_k_parameter)
        var = F(cfg_t.avst_var_parameter)
        step = int(rec[L.off_loaded + 5])
        nt = F(w.episode_time - step) / F(w.episode_time)
        res = F(mid) - F(F(F(F(inv) * gamma) * var) * nt)
        spread = F(F(F(gamma * var) * nt) + F(F(F(2) / gamma) * F(math.log(F(F(1) + F(gamma / k))))))
        spread = min(max(spread, F(tick)), F(maxint))
        bf = min(max(F(res - spread / F(2)), F(0)), F(maxint))
        af = min(max(F(res + spread / F(2)), F(0)), F(maxint))
        bp = _cvt(F(_fdiv(bf, tick) * F(tick)))
        ap = _cvt(F(_fdiv(af, tick) * F(tick)))
        rdown = (mid // tick - (1 if mid % tick == 0 else 0)) * tick
        rup = (mid // tick + 1) * tick
        return fq, fq, min(bp, rdown), max(ap, rup)
    ba, bb = (lba // tick) * tick, (lbb // tick) * tick
    if a == "spread_skew":
        mid = F(ba + bb) / F(2)
        cur = ba - bb
        stype, skew = action // 3, action % 3
        nsp = F(F(cur) * (F(1.0) if stype == 0 else F(cfg_t.spread_multiplier)))
        skt = -F(cfg_t.skew_multiplier) if skew == 0 else (F(0) if skew == 1 else F(cfg_t.skew_multiplier))
        smid = F(mid + skt * (nsp if cfg_t.multiplier_type == "spread" else F(tick)))
        hs = _fdiv(nsp, 2)
        return fq, fq, _cvt(F(_fdiv(F(smid - hs), tick) * F(tick))), _cvt(F(_fdiv(F(smid + hs), tick) * F(tick)))
    # simple
    n = 4 if cfg_t.simple_nothing_action else 3
    i = _gather(action, n)
    bo, ao = F([0, -2000, 0, 0][i]), F([0, 0, -2000, 0][i])
    if cfg_t.sell_buy_all_option:
        big = max(abs(inv), fq)
        bqa, aqa = (fq, big) if inv > 0 else (big, fq)
        bq, aq = [fq, bqa, 0, 0][i], [fq, 0, aqa, 0][i]
    else:
        bq, aq = [1, 1, 0, 0][i] * fq, [1, 0, 1, 0][i] * fq
    to = F(cfg_t.n_ticks_offset * tick)
    bp = _cvt(F(_fdiv(max(F(F(bb) - bo * to), F(0)), tick) * F(tick)))
    ap = _cvt(F(_fdiv(F(F(ba) + ao * to), tick) * F(tick)))
    return bq, aq, bp, ap


CASES = [
    dict(action_space="bobRL", bob_v0=1), dict(action_space="bobRL", bob_v0=2, fixed_quant_value=3),
    dict(action_space="bobRL", bob_v0=5), dict(action_space="bobRL", bob_v0=10),
    dict(action_space="bobStrategy", bob_v0=2), dict(action_space="bobStrategy", bob_v0=5),
    dict(action_space="AvSt"), dict(action_space="AvSt", avst_k_parameter=1.5, avst_var_parameter=2000.0),
    dict(action_space="spread_skew"),
    dict(action_space="spread_skew", multiplier_type="spread", spread_multiplier=2.0, skew_multiplier=0.5),
    dict(action_space="simple"), dict(action_space="simple", simple_nothing_action=False, n_ticks_offset=2),
    dict(action_space="simple", sell_buy_all_option=True, fixed_quant_value=2),
    dict(action_space="bobRL", bob_v0=2, fixed_action_setting=True, fixed_action=3),
]

_DAY = {}


@pytest.mark.parametrize("changes", CASES, ids=lambda d: ",".join(f"{k}={v}" for k, v in d.items()))
def test_mm_action_messages_vs_numpy(changes):
    cfg = variant(builtin_config("2_player_fq_fqc"), "MarketMaking", **changes)
    w = cfg.world_config
    if "day" not in _DAY:
        _DAY["day"] = generate_day(n_msgs=20_000, seed=5, snap_every=w.n_data_msg_per_step * w.start_resolution)
    day = _DAY["day"]
    win = make_windows(day, w)
    c, L = pack_env_cfg(cfg, len(win.starts), day.msgs.shape[0], True)
    init = O.init_states(c.lob, win, day.msgs, w, L.init_rec_words)
    E = 12
    keys = np.arange(2 * E, dtype=np.uint32).reshape(E, 2)
    st, _ = O.env_reset(c, keys, init)
    mm = cfg.dict_of_agents_configs["MarketMaking"]
    tid = w.trader_id_range_start
    checked = 0
    for k in range(6):
        for e in range(E):
            inv = int(st[e, L.agent_offsets[0] + 2])
            for act in range(-1, mm.n_actions + 1):
                rows, ex = O.mm_action_msgs(c, 0, 0, st[e], act)
                want = expected(mm, w, st[e], L, tid, act, inv)
                got = (int(rows[0, 2]), int(rows[1, 2]), int(rows[0, 3]), int(rows[1, 3]))
                assert got == want, f"step {k} env {e} action {act}: oracle {got} numpy {want}"
                assert rows[0, 0] == rows[1, 0] == 1 and rows[0, 1] == 1 and rows[1, 1] == -1
                assert rows[0, 5] == rows[1, 5] == tid
                checked += 1
        acts = O.sample_actions(c, keys + 7 * k)
        st = O.env_step(c, keys + 7 * k, acts, day.msgs, init, st)[0]
    assert checked > 100


# ------------------------------------------- MM fixed_quants / directional rows
def fixed_quant_rows(t, w, rec, L, tid, action):
    """_getActionMsgs_fixedQuant (mm_env.py:970-1118): [(type, side, qty, price)] x 2."""
    tick, nO, M = w.tick_size, w.nOrders, L.n_msgs
    asks = rec[L.off_asks:L.off_asks + 6 * nO].reshape(nO, 6)
    bids = rec[L.off_bids:L.off_bids + 6 * nO].reshape(nO, 6)
    inv = int(rec[L.agent_offsets[0] + 2])
    if t.fixed_action_setting:
        action = t.fixed_action
    ba, bb = _masked_best(asks, bids, tid, w.maxint)
    empty = ba == -1 or bb == -1
    ba, bb = (ba // tick) * tick, (bb // tick) * tick
    if empty:
        ba, bb = int(rec[L.off_best_asks + 2 * (M - 1)]), int(rec[L.off_best_bids + 2 * (M - 1)])
    fq = t.fixed_quant_value
    if not t.sell_buy_all_option:
        i = _gather(action, 10)
        bo, ao = [0, 1, 2, 3, 4, 0, 2, 5, 1, 0][i], [0, 1, 2, 3, 4, 2, 0, 1, 5, 0][i]
        bq = aq = [1] * 9 + [0]
        bq, aq = bq[i] * fq, aq[i] * fq
    else:
        i = _gather(action, 9)
        bo, ao = [10, 2, 4, -1, 0, 2, -20, 0, 0][i], [10, 2, 4, -1, 2, 0, 0, -20, 0][i]
        bq = [1, 1, 1, 1, 1, 1, inv // fq, 0, 0][i] * fq
        aq = [1, 1, 1, 1, 1, 1, 0, inv // fq, 0][i] * fq
    if empty:
        bq = aq = 0
    hsp = max(F(F(ba - bb) / F(2)), F(F(tick) / F(2)))
    hs = F(F(_fdiv(hsp, tick) + F(1)) * F(tick))
    bp = _cvt(F(_fdiv(max(F(F(bb) - F(F(bo) * hs)), F(0)), tick) * F(tick)))
    ap = _cvt(F(_fdiv(max(F(bp + tick), F(F(ba) + F(F(ao) * hs))), tick) * F(tick)))
    rows = [(1, 1, bq, bp), (1, -1, aq, ap)]
    liq = [(4, -1, int(F(t.auto_liquidate_alpha) * F(max(-inv, 0))), _cvt(F(F(ba) + F(hs * F(10))))),
           (4, 1, int(F(t.auto_liquidate_alpha) * F(max(inv, 0))), _cvt(F(F(bb) - F(hs * F(10)))))]
    if t.tenth_action == "MarketOrder" and action == 9:
        rows = liq
    if t.auto_liquidate_threshold != 0 and abs(inv) > t.auto_liquidate_threshold:
        rows = liq
    return rows


def directional_rows(t, w, rec, L, action):
    """_getActionMsgs_directional_trading (mm_env.py:1810-1865)."""
    tick, M = w.tick_size, L.n_msgs
    ba = int(rec[L.off_best_asks + 2 * (M - 1)]) // tick * tick
    bb = int(rec[L.off_best_bids + 2 * (M - 1)]) // tick * tick
    i = _gather(action, 3)
    return [(1, 1, [0, 1, 0][i] * t.fixed_quant_value, ba), (1, -1, [0, 0, 1][i] * t.fixed_quant_value, bb)]


@pytest.mark.parametrize("changes", [dict(), dict(tenth_action="NA"), dict(auto_liquidate_threshold=2),
                                     dict(sell_buy_all_option=True), dict(sell_buy_all_option=True, fixed_quant_value=2),
                                     dict(fixed_action_setting=True, fixed_action=7),
                                     dict(action_space="directional_trading", fixed_quant_value=3)],
                         ids=lambda d: ",".join(f"{k}={v}" for k, v in d.items()) or "metric")
def test_mm_fixed_quant_and_directional_vs_numpy(changes):
    cfg = variant(builtin_config("2_player_fq_fqc"), "MarketMaking", **changes)
    w = cfg.world_config
    if "day" not in _DAY:
        _DAY["day"] = generate_day(n_msgs=20_000, seed=5, snap_every=w.n_data_msg_per_step * w.start_resolution)
    day = _DAY["day"]
    win = make_windows(day, w)
    c, L = pack_env_cfg(cfg, len(win.starts), day.msgs.shape[0], True)
    init = O.init_states(c.lob, win, day.msgs, w, L.init_rec_words)
    E = 12
    keys = np.arange(2 * E, dtype=np.uint32).reshape(E, 2) + 5
    st, _ = O.env_reset(c, keys, init)
    mm = cfg.dict_of_agents_configs["MarketMaking"]
    tid = w.trader_id_range_start
    liq = 0
    for k in range(8):
        for e in range(E):
            for act in range(-1, mm.n_actions + 1):
                rows, _ = O.mm_action_msgs(c, 0, 0, st[e], act)
                want = (directional_rows(mm, w, st[e], L, act) if mm.action_space == "directional_trading"
                        else fixed_quant_rows(mm, w, st[e], L, tid, act))
                got = [tuple(int(v) for v in r[:4]) for r in rows]
                assert got == want, f"step {k} env {e} action {act}: oracle {got} numpy {want}"
                liq += got[0][0] == 4
        acts = O.sample_actions(c, keys + 7 * k)
        st = O.env_step(c, keys + 7 * k, acts, day.msgs, init, st)[0]
    if mm.action_space == "fixed_quants" and mm.tenth_action == "MarketOrder" and not mm.fixed_action_setting:
        assert liq > 0


# ------------------------------------------------------------ MM observations
def mm_obs_numpy(t, w, rec, L, a_off):
    """_get_obs_basic (mm_env.py:2963-3000) / _get_obs_engineered (:3004-3154), normalize_obs
    (:3157-3167), ravel_pytree key order, from the record the step produced."""
    M = L.n_msgs
    pa = int(rec[L.off_best_asks + 2 * (M - 1)])
    pb = int(rec[L.off_best_bids + 2 * (M - 1)])
    spread = abs(pa - pb)
    inv = int(rec[a_off + 2])
    if t.observation_space == "basic":
        obs, std = {"inventory": inv, "spread": spread}, {"inventory": 10, "spread": 1e4}
    else:
        asks = rec[L.off_asks:L.off_asks + 6 * w.nOrders].reshape(-1, 6)
        bids = rec[L.off_bids:L.off_bids + 6 * w.nOrders].reshape(-1, 6)
        wr = rec[L.off_world:L.off_world + 5]
        lr = rec[L.off_loaded:L.off_loaded + 6]
        obs = {"p_bid": pb, "p_ask": pa, "spread": spread,
               "q_bid": int(np.where(bids[:, 0] != -1, bids[:, 1], 0).sum()),
               "q_ask": int(np.where(asks[:, 0] != -1, asks[:, 1], 0).sum()),
               "mid_price": wr[3:4].view(np.float32)[0], "step_counter": int(lr[5]), "inventory": inv}
        std = {"p_bid": 1e6, "p_ask": 1e6, "spread": 1e4, "q_bid": 1000, "q_ask": 1000, "mid_price": 1e6,
               "step_counter": 10, "inventory": 10}
        if w.ep_type == "fixed_time":
            time = F(F(wr[0]) + F(wr[1]) / F(1e9))
            elapsed = F(time - F(F(lr[0]) + F(lr[1]) / F(1e9)))
            obs.update(delta_time=wr[4:5].view(np.float32)[0], time_remaining=F(F(w.episode_time) - elapsed))
            std.update(delta_time=10, time_remaining=w.episode_time)
    keys = sorted(obs)
    if t.normalize:
        return [F(F(obs[k]) / F(std[k])) for k in keys]
    return [F(obs[k]) for k in keys]


@pytest.mark.parametrize("obs_space,norm,ep", [("basic", True, "fixed_steps"), ("engineered", True, "fixed_steps"),
                                               ("engineered", False, "fixed_steps"),
                                               ("engineered", True, "fixed_time"), ("engineered", False, "fixed_time")])
def test_mm_obs_vs_numpy(obs_space, norm, ep, tmp_path):
    cfg = variant(builtin_config("2_player_fq_fqc"), "MarketMaking", observation_space=obs_space, normalize=norm)
    if ep == "fixed_time":
        import dataclasses
        from hftlob.data import lobster as Lb
        from hftlob.data.raw_synthetic import write_raw_lobster_day
        w = dataclasses.replace(cfg.world_config, ep_type="fixed_time", episode_time=300, start_resolution=300)
        cfg = dataclasses.replace(cfg, world_config=w)
        write_raw_lobster_day(str(tmp_path), n_events=12_000, seed=3, mid=2_000_000)
        ld = Lb.LoadLOBSTER_resample(str(tmp_path), str(tmp_path), 10, "fixed_time", window_length=300,
                                     window_resolution=300, n_data_msg_per_step=100, stock="SYN",
                                     time_period="2026_Oct")
        day = Lb.LoadedDay.from_arrays(*ld.run_loading("cpu_ft"))
    else:
        w = cfg.world_config
        day = generate_day(n_msgs=20_000, seed=6, snap_every=w.n_data_msg_per_step * w.start_resolution)
    w = cfg.world_config
    t = cfg.dict_of_agents_configs["MarketMaking"]
    win = make_windows(day, w)
    c, L = pack_env_cfg(cfg, len(win.starts), day.msgs.shape[0], True)
    init = O.init_states(c.lob, win, day.msgs, w, L.init_rec_words)
    E = 8
    keys = np.arange(2 * E, dtype=np.uint32).reshape(E, 2)
    st, o = O.env_reset(c, keys, init)
    d = L.obs_dims[0]
    assert d == {"basic": 2, "engineered": 8 if ep == "fixed_steps" else 10}[obs_space]
    for k in range(12):
        for e in range(E):
            want = mm_obs_numpy(t, w, st[e], L, L.agent_offsets[0])
            assert np.array_equal(o[e, 0, :d], np.array(want, np.float32)), (k, e, o[e, 0, :d], want)
        acts = O.sample_actions(c, keys + 3 * k)
        st, o = O.env_step(c, keys + 3 * k, acts, day.msgs, init, st)[:2]
