"""Engine parity: HIP hftlob_book_process vs the CPU oracle, bit-exact (int32)."""
import zlib

import numpy as np
import pytest
import torch

from hftlob.config import JAXLOB_Configuration
from hftlob.engine import book_process_, scan_through_entire_array_save_bidask
from hftlob.layout import pack_lob_cfg
from oracle import pyoracle as O
from streams import (full_book_messages, init_book_messages, neg1_trade_streams, noop_streams, odd_add_streams,
                     random_streams, top_streams)

pytestmark = pytest.mark.gpu

CASES = [
    dict(),                                                    # metric config engine settings
    dict(type_4_interpretation=1),                              # LIM
    dict(type_4_interpretation=2),                              # MKT
    dict(check_book_fill=False),
    dict(cancel_mode=0),
    dict(nOrders=16, nTrades=8),                                # book-full eviction + trade overwrite
    dict(nOrders=40, nTrades=30, type_4_interpretation=1),
    dict(nOrders=200, nTrades=150),                             # 4 slot sets per lane
    dict(cancel_mode=2),                                        # random cancel fallback (:141-155)
    dict(cancel_mode=3),                                        # + random large (:157-164)
    dict(cancel_mode=3, nOrders=40, nTrades=30, _legacy=True),  # legacy threefry split / bits
    dict(cancel_mode=2, nOrders=200, nTrades=150),
]


def _run(cfg, msgs, a0, b0, t0, part=True):
    lc = pack_lob_cfg(cfg, part)
    E = msgs.shape[0]
    keys = np.random.default_rng(E + msgs.shape[1]).integers(0, 2**32, (E, 2), dtype=np.uint64).astype(np.uint32)
    oa, ob, ot, oba, obb = O.book_process(lc, msgs, a0, b0, t0, keys=keys)
    dev = "cuda"
    ga, gb, gt = (torch.from_numpy(x.copy()).to(dev) for x in (a0, b0, t0))
    gba = torch.empty((msgs.shape[0], msgs.shape[1], 2), dtype=torch.int32, device=dev)
    gbb = torch.empty_like(gba)
    book_process_(cfg, torch.from_numpy(msgs).to(dev), ga, gb, gt, gba, gbb,
                  keys=torch.from_numpy(keys.view(np.int32)).to(dev), prng_partitionable=part)
    torch.cuda.synchronize()
    for name, o, g in (("asks", oa, ga), ("bids", ob, gb), ("trades", ot, gt), ("best_asks", oba, gba),
                       ("best_bids", obb, gbb)):
        g = g.cpu().numpy()
        bad = np.argwhere(o != g)
        assert bad.size == 0, f"{name} mismatch at {bad[:5].tolist()}: oracle {o[tuple(bad[0])]} gpu {g[tuple(bad[0])]}"


@pytest.mark.parametrize("kw", CASES, ids=[str(k) or "default" for k in CASES])
def test_book_random_streams(kw):
    kw = dict(kw)
    part = not kw.pop("_legacy", False)
    cfg = JAXLOB_Configuration(**kw)
    E, M = 48, 300
    init = init_book_messages(E, seed=1)
    empty_a = np.full((E, cfg.nOrders, 6), -1, np.int32)
    empty_t = np.full((E, cfg.nTrades, 8), -1, np.int32)
    a0, b0, t0, _, _ = O.book_process(pack_lob_cfg(cfg), init, empty_a, empty_a, empty_t, save_best=False)
    msgs = random_streams(E, M, seed=zlib.crc32(str(sorted(kw.items())).encode()) % 1000)
    _run(cfg, msgs, a0, b0, empty_t, part)
    # and from empty books, with a non-empty incoming trade log
    _run(cfg, msgs, empty_a, empty_a, t0, part)


def test_book_functional_api():
    cfg = JAXLOB_Configuration()
    msgs = torch.from_numpy(random_streams(1, 50, seed=3)[0]).cuda()
    a = torch.full((100, 6), -1, dtype=torch.int32).cuda()
    (na, nb, nt), (ba, bb) = scan_through_entire_array_save_bidask(cfg, None, msgs, (a, a, torch.full((100, 8), -1, dtype=torch.int32).cuda()), 10)
    assert ba.shape == (10, 2) and (a == -1).all()   # inputs untouched, last N rows returned


def test_book_empty_and_max_sizes():
    """n_env = 0 and n_msg = 0 are no-ops; nOrders = nTrades = 256 (HFTLOB_MAX_SLOTS) is parity-exact."""
    cfg = JAXLOB_Configuration()
    a = torch.full((0, 100, 6), -1, dtype=torch.int32, device="cuda")
    t = torch.full((0, 100, 8), -1, dtype=torch.int32, device="cuda")
    book_process_(cfg, torch.empty((0, 5, 8), dtype=torch.int32, device="cuda"), a, a.clone(), t)
    a1 = torch.full((3, 100, 6), -1, dtype=torch.int32, device="cuda")
    a1[:, 0] = torch.tensor([200, 5, 1, 1, 0, 0], dtype=torch.int32)
    before = a1.clone()
    t1 = torch.full((3, 100, 8), -1, dtype=torch.int32, device="cuda")
    book_process_(cfg, torch.empty((3, 0, 8), dtype=torch.int32, device="cuda"), a1, a1.clone(), t1)
    torch.cuda.synchronize()
    assert torch.equal(a1, before) and (t1 == -1).all()
    big = JAXLOB_Configuration(nOrders=256, nTrades=256)
    E, M = 8, 400
    init = init_book_messages(E, seed=4)
    empty_a = np.full((E, 256, 6), -1, np.int32)
    empty_t = np.full((E, 256, 8), -1, np.int32)
    a0, b0, _, _, _ = O.book_process(pack_lob_cfg(big), init, empty_a, empty_a, empty_t, save_best=False)
    _run(big, random_streams(E, M, seed=77), a0, b0, empty_t)


@pytest.mark.parametrize("kw", [dict(), dict(nOrders=16, nTrades=8), dict(type_4_interpretation=1),
                                dict(type_4_interpretation=2)], ids=["default", "nO16", "t4lim", "t4mkt"])
def test_book_odd_adds(kw):
    """Adds priced <= 0 or maxint and add-kind messages whose side is not -1 / 1
    (streams.odd_add_streams): the decode marks them RARE, the general handlers take them, and
    the common handlers that follow see the book they left (negative-price rows, full sides)."""
    cfg = JAXLOB_Configuration(**kw)
    E, M = 64, 400
    init = init_book_messages(E, seed=6)
    empty_a = np.full((E, cfg.nOrders, 6), -1, np.int32)
    empty_t = np.full((E, cfg.nTrades, 8), -1, np.int32)
    a0, b0, _, _, _ = O.book_process(pack_lob_cfg(cfg), init, empty_a, empty_a, empty_t, save_best=False)
    msgs = odd_add_streams(E, M, seed=31 + cfg.nOrders)
    _run(cfg, msgs, a0, b0, empty_t)
    _run(cfg, msgs, empty_a, empty_a, empty_t)


@pytest.mark.parametrize("kw", [dict(), dict(nOrders=16, nTrades=8), dict(type_4_interpretation=1)],
                         ids=["default", "nO16", "t4lim"])
def test_book_top_of_book_cache(kw):
    """Crossing-heavy streams with tied and out-of-order times (streams.top_streams): every match
    trip's top-of-book slot equals the oracle's (this stream caught a top-of-book slot cache that
    the metric's and the random streams did not)."""
    cfg = JAXLOB_Configuration(**kw)
    E, M = 64, 400
    init = init_book_messages(E, seed=5)
    empty_a = np.full((E, cfg.nOrders, 6), -1, np.int32)
    empty_t = np.full((E, cfg.nTrades, 8), -1, np.int32)
    a0, b0, _, _, _ = O.book_process(pack_lob_cfg(cfg), init, empty_a, empty_a, empty_t, save_best=False)
    msgs = top_streams(E, M, seed=11 + cfg.nOrders)
    _run(cfg, msgs, a0, b0, empty_t)
    _run(cfg, msgs, empty_a, empty_a, empty_t)


@pytest.mark.parametrize("kw", [dict(), dict(nOrders=16, nTrades=8), dict(nOrders=40, nTrades=30)],
                         ids=["default", "nO16_nT8", "nO40_nT30"])
def test_book_trade_row_neg1_fields(kw):
    """Crossing messages with oid == -1 or time == -1 (streams.neg1_trade_streams): the trade log's
    next row is the first whose col 4 (the trade's TIME) is -1 (JaxOrderBookArrays.py:205), so
    a time == -1 trade is overwritten by the next one and an oid == -1 trade is kept."""
    cfg = JAXLOB_Configuration(**kw)
    E, M = 64, 400
    init = init_book_messages(E, seed=6)
    empty_a = np.full((E, cfg.nOrders, 6), -1, np.int32)
    empty_t = np.full((E, cfg.nTrades, 8), -1, np.int32)
    a0, b0, _, _, _ = O.book_process(pack_lob_cfg(cfg), init, empty_a, empty_a, empty_t, save_best=False)
    msgs = neg1_trade_streams(E, M, seed=21 + cfg.nOrders)
    assert ((msgs[..., 4] == -1) & (msgs[..., 0] == 4)).any() and ((msgs[..., 6] == -1) & (msgs[..., 0] == 4)).any()
    _run(cfg, msgs, a0, b0, empty_t)
    _run(cfg, msgs, empty_a, empty_a, empty_t)


def test_book_top_of_book_cache_4096():
    """The top-of-book stress stream at the metric's size (4096 envs, 100 slots): the cached
    top-of-book slot of each side against the oracle's formula on every crossing message."""
    cfg = JAXLOB_Configuration()
    E, M = 4096, 400
    init = init_book_messages(E, seed=8)
    empty_a = np.full((E, cfg.nOrders, 6), -1, np.int32)
    empty_t = np.full((E, cfg.nTrades, 8), -1, np.int32)
    a0, b0, _, _, _ = O.book_process(pack_lob_cfg(cfg), init, empty_a, empty_a, empty_t, save_best=False)
    _run(cfg, top_streams(E, M, seed=13), a0, b0, empty_t)


NOOP_CASES = [dict(), dict(nOrders=16, nTrades=8), dict(nOrders=40, nTrades=30), dict(type_4_interpretation=1),
              dict(cancel_mode=0), dict(cancel_mode=2), dict(nOrders=200, nTrades=150)]


@pytest.mark.parametrize("kw", NOOP_CASES, ids=[str(k) or "default" for k in NOOP_CASES])
def test_book_noop_skip(kw):
    """The chunk pre-pass that skips messages leaving the book unchanged (streams.noop_streams:
    unmatched cancels wrapping to the last slot, zero / -1 / negative quantities, doNothing rows,
    init-id rows and adds, -1 fields) over books whose sides are 85-100 % full (the last slot
    occupied or not, a few free rows) and over empty books: books, trades and every message's
    best-quote record bit-exact."""
    cfg = JAXLOB_Configuration(**kw)
    E, M = 96, 320
    empty_a = np.full((E, cfg.nOrders, 6), -1, np.int32)
    empty_t = np.full((E, cfg.nTrades, 8), -1, np.int32)
    init = full_book_messages(E, seed=9, nO=cfg.nOrders)
    a0, b0, _, _, _ = O.book_process(pack_lob_cfg(cfg), init, empty_a, empty_a, empty_t, save_best=False)
    msgs = noop_streams(E, M, seed=31 + cfg.nOrders + 7 * cfg.cancel_mode, nO=cfg.nOrders)
    _run(cfg, msgs, a0, b0, empty_t)
    _run(cfg, msgs, empty_a, empty_a, empty_t)
