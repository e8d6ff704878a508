"""Pin the oracles before trusting them: hand-derived golden scenarios, the
reference's own smoke inputs (jorderbook.py __main__), Random123 KATs, the
documented JAX split value, and C-oracle vs numpy-oracle agreement."""
import numpy as np
import pytest

from golden.book_scenarios import (JORDERBOOK_EXPECT, JORDERBOOK_MSGS, SCENARIOS, jorderbook_init_msgs)
from hftlob.config import JAXLOB_Configuration
from hftlob.layout import pack_lob_cfg
from oracle import pyoracle as O
from oracle import ref_py as R
from streams import init_book_messages, random_streams


def _expand(rows_by_idx, n, width):
    out = np.full((n, width), -1, np.int32)
    for i, r in rows_by_idx.items():
        out[i] = r
    return out


@pytest.mark.parametrize("name", sorted(SCENARIOS))
def test_golden_scenarios_c_oracle(name):
    sc = SCENARIOS[name]
    cfg = JAXLOB_Configuration(**sc["cfg"])
    msgs = np.array([sc["msgs"]], np.int32)
    a, b, t, ba, bb = O.book_process(pack_lob_cfg(cfg), msgs, np.array([sc["asks"]], np.int32),
                                     np.array([sc["bids"]], np.int32),
                                     np.full((1, cfg.nTrades, 8), -1, np.int32))
    assert a[0].tolist() == sc["exp_asks"]
    assert b[0].tolist() == sc["exp_bids"]
    assert t[0].tolist() == _expand(sc["exp_trades"], cfg.nTrades, 8).tolist()
    assert ba[0].tolist() == sc["exp_best_asks"]
    assert bb[0].tolist() == sc["exp_best_bids"]


@pytest.mark.parametrize("name", sorted(SCENARIOS))
def test_golden_scenarios_numpy_oracle(name):
    sc = SCENARIOS[name]
    cfg = R.default_cfg(**sc["cfg"])
    (a, b, t), ba, bb = R.scan_save_bidask(cfg, sc["msgs"], sc["asks"], sc["bids"],
                                           np.full((cfg["nTrades"], 8), -1, np.int32))
    assert a.tolist() == sc["exp_asks"] and b.tolist() == sc["exp_bids"]
    assert t.tolist() == _expand(sc["exp_trades"], cfg["nTrades"], 8).tolist()
    assert ba.tolist() == sc["exp_best_asks"] and bb.tolist() == sc["exp_best_bids"]


def test_jorderbook_reference_inputs():
    cfg = JAXLOB_Configuration()
    msgs = np.array([jorderbook_init_msgs() + JORDERBOOK_MSGS], np.int32)
    e = np.full((1, 100, 6), -1, np.int32)
    a, b, t, ba, bb = O.book_process(pack_lob_cfg(cfg), msgs, e, e, np.full((1, 100, 8), -1, np.int32))
    for i, r in JORDERBOOK_EXPECT["bids_rows"].items():
        assert b[0, i].tolist() == r
    for i, r in JORDERBOOK_EXPECT["asks_rows"].items():
        assert a[0, i].tolist() == r
    for i, r in JORDERBOOK_EXPECT["trades_rows"].items():
        assert t[0, i].tolist() == r
    assert ba[0, -2:].tolist() == JORDERBOOK_EXPECT["best_asks"]
    assert bb[0, -2:].tolist() == JORDERBOOK_EXPECT["best_bids"]


KATS = [((0, 0), (0, 0), (0x6B200159, 0x99BA4EFE)),
        ((0xFFFFFFFF, 0xFFFFFFFF), (0xFFFFFFFF, 0xFFFFFFFF), (0x1CB996FC, 0xBB002BE7)),
        ((0x13198A2E, 0x03707344), (0x243F6A88, 0x85A308D3), (0xC4923A9C, 0x483DF7A0))]


@pytest.mark.parametrize("key,ctr,out", KATS)
def test_threefry_random123_kat(key, ctr, out):
    assert O.threefry2x32(key[0], key[1], ctr[0], ctr[1]) == out
    assert R.threefry2x32(key[0], key[1], ctr[0], ctr[1]) == out


def test_jax_documented_legacy_split():
    # jax.random.split(PRNGKey(0)) with jax_threefry_partitionable=False (JAX docs)
    want = [[4146024105, 967050713], [2718843009, 1272950319]]
    assert O.split_keys([[0, 0]], 2, partitionable=False)[0].tolist() == want
    assert [list(k) for k in R.split((0, 0), 2, partitionable=False)] == want


@pytest.mark.parametrize("part", [True, False])
def test_prng_c_vs_numpy(part):
    rng = np.random.default_rng(5)
    for _ in range(50):
        k = [int(x) for x in rng.integers(0, 2**32, 2, dtype=np.uint64)]
        n = int(rng.integers(1, 7))
        assert O.split_keys([k], n, part)[0].tolist() == [list(x) for x in R.split(k, n, part)]
        hi = int(rng.integers(1, 1000))
        assert O.randint(k, 0, hi, part) == R.randint(k, 0, hi, part)


@pytest.mark.parametrize("kw", [dict(), dict(type_4_interpretation=1), dict(type_4_interpretation=2),
                                dict(nOrders=12, nTrades=6), dict(check_book_fill=False, nOrders=20)])
def test_c_oracle_vs_numpy_oracle_random(kw):
    cfg = JAXLOB_Configuration(**kw)
    rc = R.default_cfg(**kw)
    E, M = 6, 120
    init = init_book_messages(E, seed=2)
    msgs = random_streams(E, M, seed=9)
    full = np.concatenate([init, msgs], axis=1)
    e6 = np.full((E, cfg.nOrders, 6), -1, np.int32)
    e8 = np.full((E, cfg.nTrades, 8), -1, np.int32)
    a, b, t, ba, bb = O.book_process(pack_lob_cfg(cfg), full, e6, e6, e8)
    for i in range(E):
        (ra, rb, rt), rba, rbb = R.scan_save_bidask(rc, full[i], e6[i], e6[i], e8[i])
        assert (ra == a[i]).all() and (rb == b[i]).all() and (rt == t[i]).all()
        assert (rba == ba[i]).all() and (rbb == bb[i]).all()


@pytest.mark.parametrize("mode,part", [(2, True), (3, True), (3, False)])
def test_c_oracle_vs_numpy_oracle_random_cancel(mode, part):
    """cancel_mode 2/3 (get_random_id_match / get_random_large_id_match): C vs numpy restatement."""
    cfg = JAXLOB_Configuration(cancel_mode=mode)
    rc = R.default_cfg(cancel_mode=mode, partitionable=part)
    E, M = 6, 160
    init = init_book_messages(E, seed=4)
    msgs = random_streams(E, M, seed=21)
    full = np.concatenate([init, msgs], axis=1)
    e6 = np.full((E, cfg.nOrders, 6), -1, np.int32)
    e8 = np.full((E, cfg.nTrades, 8), -1, np.int32)
    keys = np.random.default_rng(mode).integers(0, 2**32, (E, 2), dtype=np.uint64).astype(np.uint32)
    a, b, t, ba, bb = O.book_process(pack_lob_cfg(cfg, part), full, e6, e6, e8, keys=keys)
    a1, b1, _, _, _ = O.book_process(pack_lob_cfg(JAXLOB_Configuration(cancel_mode=1)), full, e6, e6, e8)
    assert (a1 != a).any() or (b1 != b).any(), "the random fallback never changed the book"
    for i in range(E):
        (ra, rb, rt), rba, rbb = R.scan_save_bidask(rc, full[i], e6[i], e6[i], e8[i], key=tuple(int(x) for x in keys[i]))
        assert (ra == a[i]).all() and (rb == b[i]).all() and (rt == t[i]).all()
        assert (rba == ba[i]).all() and (rbb == bb[i]).all()


def test_random_cancel_choice_semantics():
    """Hand-derived: with one price-matched order the draw must pick it, whatever the key;
    with none, chosen id is 0 and the -1 index wraps to the last slot."""
    cfg = R.default_cfg(cancel_mode=2, nOrders=4)
    side = np.full((4, 6), -1, np.int32)
    side[0] = [100, 5, 77, 1, 0, 0]
    side[2] = [101, 9, 55, 1, 0, 0]
    msg = dict(price=101, quantity=3, orderid=999)
    for k in range(20):
        assert R.get_random_id_match(cfg, (k, 3 * k + 1), side, msg) == 2
    msg = dict(price=102, quantity=3, orderid=999)
    assert R.get_random_id_match(cfg, (1, 2), side, msg) == -1
    out = R.cancel_order(cfg, side, msg, key=(1, 2))
    assert (out[3] == -1).all() and (out[:3] == side[:3]).all()   # slot -1 (empty) -> stays removed
