"""The message-skip predicate of the HIP kernels (hftlob.hip chunk_noops), restated in numpy and
checked against the C oracle message by message: every message the predicate marks as a no-op,
decided from the book at its chunk's start, must leave the oracle's book and trade log unchanged,
and the predicate must fire on the streams aimed at it (tests/streams.py noop_streams), at the
room boundary too.  CPU only; the GPU parity tests (test_gpu_book.py::test_book_noop_skip and
every env test) check the kernels themselves."""
import numpy as np
import pytest

from hftlob.config import JAXLOB_Configuration
from hftlob.layout import pack_lob_cfg
from oracle import pyoracle as O
from streams import full_book_messages, noop_streams, random_streams

M32 = 0xFFFFFFFF
H_ASK, H_BID, H_CNL_ASK, H_CNL_BID, H_NOP = 0, 1, 2, 3, 4


def hash_id(v):
    return ((int(v) & M32) * 0x9E3779B1 & M32) >> 21


def hash_px(p, ask):
    return (((int(p) & M32) * 0x85EBCA6B & M32) ^ (0xC2B2AE35 if ask else 0x27D4EB2F)) >> 21


def decode(m, t4):
    """decode_msgs (hftlob.hip; cond_type_side_save_bidask, JaxOrderBookArrays.py:687-732):
    (kind, neg1_or_pm1 flag of an add)."""
    ty, sd = int(m[0]), int(m[1])
    if ty == 4:
        sd = -sd
    cnl = ty in (2, 3)
    h = H_ASK
    if ty == 0 and sd == 0:
        h = H_NOP
    if ty in (1, 4) and sd == 1:
        h = H_BID
    if cnl and sd == 1:
        h = H_CNL_BID
    if cnl and sd == -1:
        h = H_CNL_ASK
    p_add = (2**31 - 1 if h == H_BID else 0) if t4 == 2 else int(m[3])
    flag = (p_add != -1 and (-1 in (int(m[4]), int(m[5]), int(m[6]), int(m[7])))) or p_add == -1
    return h, flag


def fast(a, b):
    """The books in which the kernels may run the FAST variant (hftlob.hip F_FAST): both sides
    clean (a row with q <= 0 is all -1), no row with p != -1 holding a -1, and a p == -1 row all -1
    but possibly q (a FAST cancel of a negative quantity can leave q > 0 there).  A superset of
    the kernels' FAST states, so the emulation skips at least where they do."""
    for s in (a, b):
        allm1 = (s == -1).all(1)
        if ((s[:, 1] <= 0) & ~allm1).any():
            return False
        if ((s[:, 0] != -1) & (s == -1).any(1)).any():
            return False
        if ((s[:, 0] == -1) & (s[:, [2, 3, 4, 5]] != -1).any(1)).any():
            return False
    return True


def noops(cfg, a, b, chunk):
    """chunk_noops: the chunk's skippable messages, from the book (a, b) at the chunk's start."""
    n, R = len(chunk), cfg.nOrders
    dec = [decode(m, cfg.type_4_interpretation) for m in chunk]
    kind = np.array([d[0] for d in dec])
    skip = kind == H_NOP
    if not fast(a, b):
        return skip
    lo = cfg.init_id - 2 * cfg.book_depth
    span = cfg.init_id - lo
    initr = lambda o: 0 <= ((int(o) - lo) & M32) <= span  # noqa: E731
    qty, price, oid = chunk[:, 2], chunk[:, 3], chunk[:, 4]
    cnl = (kind == H_CNL_ASK) | (kind == H_CNL_BID)
    add = (kind == H_ASK) | (kind == H_BID)
    brk = [(add[k] and (dec[k][1] or initr(oid[k]))) or (cnl[k] and qty[k] < -1) for k in range(n)]
    first = brk.index(True) if any(brk) else n
    before = np.arange(n) < first
    skip = skip | (cnl & (qty == 0) & before)
    if cfg.cancel_mode >= 2 or initr(-1):
        return skip
    bits = set()
    for sd, s in ((True, a), (False, b)):
        for r in s:
            if r[2] != -1:
                bits.add(hash_id(r[2]))
            if initr(r[2]):
                bits.add(hash_px(r[0], sd))
    for k in range(n):
        if add[k]:
            bits.add(hash_id(oid[k]))

    def room(s):
        if not (s[R - 1, 0] == -1 and s[R - 1, 1] == -1):
            return -1
        return int((s[:R - 1, 0] == -1).sum())

    ra, rb = room(a), room(b)
    na = nb = 0
    for k in range(n):
        if cnl[k] and before[k] and qty[k] >= -1 and oid[k] != -1:
            ask = kind[k] == H_CNL_ASK
            hit = hash_id(oid[k]) in bits or hash_px(price[k], ask) in bits
            rm, nadd = (ra, na) if ask else (rb, nb)
            if not hit and rm >= 0 and nadd <= rm:
                skip[k] = True
        na += kind[k] == H_ASK
        nb += kind[k] == H_BID
    return skip


def _check(cfg, msgs, a0, b0, t0):
    lc = pack_lob_cfg(cfg)
    n_skip = n_room_edge = 0
    for e in range(msgs.shape[0]):
        a, b, t = a0[e:e + 1].copy(), b0[e:e + 1].copy(), t0[e:e + 1].copy()
        for base in range(0, msgs.shape[1], 64):
            chunk = msgs[e, base:base + 64]
            sk = noops(cfg, a[0], b[0], chunk)
            for k in range(len(chunk)):
                a1, b1, t1, _, _ = O.book_process(lc, chunk[None, k:k + 1], a, b, t, save_best=False)
                if sk[k]:
                    assert (a1 == a).all() and (b1 == b).all() and (t1 == t).all(), \
                        f"env {e} msg {base + k} {chunk[k].tolist()} marked a no-op but changes the book"
                    n_skip += 1
                    free_a = int((a[0, :-1, 0] == -1).sum())
                    free_b = int((b[0, :-1, 0] == -1).sum())
                    n_room_edge += min(free_a, free_b) <= 2
                a, b, t = a1, b1, t1
    return n_skip, n_room_edge


@pytest.mark.parametrize("kw", [dict(), dict(nOrders=16, nTrades=8), dict(type_4_interpretation=1),
                                dict(cancel_mode=2)], ids=["default", "nO16", "t4lim", "cm2"])
def test_noop_predicate_is_exact(kw):
    cfg = JAXLOB_Configuration(**kw)
    E, M = 6, 192
    empty_a = np.full((E, cfg.nOrders, 6), -1, np.int32)
    empty_t = np.full((E, cfg.nTrades, 8), -1, np.int32)
    init = full_book_messages(E, seed=9, nO=cfg.nOrders)
    a0, b0, _, _, _ = O.book_process(pack_lob_cfg(cfg), init, empty_a, empty_a, empty_t, save_best=False)
    msgs = noop_streams(E, M, seed=31 + cfg.nOrders + 7 * cfg.cancel_mode, nO=cfg.nOrders)
    n1, edge = _check(cfg, msgs, a0, b0, empty_t)
    n2, _ = _check(cfg, msgs, empty_a, empty_a, empty_t)
    n3, _ = _check(cfg, random_streams(E, M, seed=5), a0, b0, empty_t)
    assert n1 + n2 > E * M // 10, (n1, n2)   # the stream exercises the skip
    if cfg.cancel_mode < 2:
        assert edge > 0                      # ... with nearly full sides
