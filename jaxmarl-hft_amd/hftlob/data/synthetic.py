"""Seeded synthetic LOBSTER trading day, in the reference's post-load layout.

No LOBSTER data ships with the reference or this image, so the benchmark and
the tests replay a generated day.  The generator keeps a full-depth L3 book
and emits the message mix of a liquid NASDAQ name, with LOBSTER semantics:

* message rows are ``[type, direction, qty, price, trader_id(=order id),
  order_id, time_s, time_ns]`` int32 — the column order and type recoding of
  ``LoadLOBSTER_resample._pre_process_msg_ob`` / ``_get_inits_day``
  (``jaxlobster/lobster_loader.py:891-945, 1004-1071``): types 1 (limit),
  2 (partial cancel and, after recoding, 3 = delete), 4 (execution of a
  standing order; ``direction`` is the standing order's side);
* ids of cancels / executions refer to live orders; executions hit the front
  of the best level (price-time priority); ~5 % of limits are marketable;
* 10-level snapshots ``[ask_p1, ask_q1, bid_p1, bid_q1, ...]`` taken before a
  window's first message (the loader's one-row book/message alignment shift);
  empty levels carry LOBSTER's +/-9999999999 prices wrapped to int32, size 0.

Two price regimes: ``mid=2_000_000`` (AMZN-2024-like, exact in float32) and
``mid=28_000_000`` (GOOG-2022-like, above 2**24, exercises f32 rounding).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
from sortedcontainers import SortedDict

EMPTY_ASK = np.int64(9999999999).astype(np.int32)    # int64 -> int32 wrap, as jnp.asarray does
EMPTY_BID = np.int64(-9999999999).astype(np.int32)


@dataclass
class LobsterDay:
    msgs: np.ndarray          # (N, 8) int32
    books: np.ndarray         # (N_snap, 40) int32 — snapshot BEFORE message i at snap_idx[i]
    snap_idx: np.ndarray      # message indices of the snapshots
    tick_size: int


def generate_day(n_msgs: int = 400_000, seed: int = 20260403, mid: int = 2_000_000, tick: int = 100,
                 snap_every: int = 6400, levels: int = 10, day_start: int = 34200, day_end: int = 57600) -> LobsterDay:
    rng = np.random.Generator(np.random.PCG64(seed))
    asks, bids = SortedDict(), SortedDict()       # price -> list of [oid, qty]
    where = {}                                    # oid -> (side, price)
    next_oid = 10_000_000

    def add(side, price, qty):
        nonlocal next_oid
        oid = next_oid
        next_oid += 1
        book = bids if side == 1 else asks
        book.setdefault(price, []).append([oid, qty])
        where[oid] = (side, price)
        return oid

    def remove_qty(oid, qty):
        side, price = where[oid]
        book = bids if side == 1 else asks
        lvl = book[price]
        for k, (o, q) in enumerate(lvl):
            if o == oid:
                if q - qty <= 0:
                    lvl.pop(k)
                    del where[oid]
                else:
                    lvl[k][1] = q - qty
                break
        if not lvl:
            del book[price]

    picker = _LivePicker(where, rng)
    for k in range(1, 21):                      # seed book: 20 levels a side
        for _ in range(int(rng.integers(1, 5))):
            add(-1, mid + k * tick, int(max(1, round(rng.lognormal(4.0, 1.0)))))
            add(1, mid - k * tick, int(max(1, round(rng.lognormal(4.0, 1.0)))))

    msgs = np.zeros((n_msgs, 8), dtype=np.int64)
    n_snap = (n_msgs + snap_every - 1) // snap_every
    books = np.zeros((n_snap, 4 * levels), dtype=np.int64)
    snap_idx = np.arange(n_snap) * snap_every
    # time grid: strictly increasing (s, ns) spread over the trading day
    span_ns = (day_end - day_start) * 1_000_000_000
    gaps = rng.exponential(1.0, n_msgs)
    t_ns = np.cumsum(gaps / gaps.sum() * (span_ns * 0.999)).astype(np.int64) + np.arange(n_msgs)
    u = rng.random(n_msgs)
    side_draw = rng.integers(0, 2, n_msgs) * 2 - 1
    geo = rng.geometric(0.35, n_msgs) - 1
    lqty = np.maximum(1, np.round(rng.lognormal(4.0, 1.0, n_msgs))).astype(np.int64)
    pick = rng.random(n_msgs)
    mkt = rng.random(n_msgs)

    def snapshot(row):
        a_lv, b_lv = list(asks.items())[:levels], list(reversed(bids.items()))[:levels]
        for k in range(levels):
            if k < len(a_lv):
                books[row, 4 * k] = a_lv[k][0]
                books[row, 4 * k + 1] = sum(q for _, q in a_lv[k][1])
            else:
                books[row, 4 * k] = EMPTY_ASK
            if k < len(b_lv):
                books[row, 4 * k + 2] = b_lv[k][0]
                books[row, 4 * k + 3] = sum(q for _, q in b_lv[k][1])
            else:
                books[row, 4 * k + 2] = EMPTY_BID

    for i in range(n_msgs):
        if i % snap_every == 0:
            snapshot(i // snap_every)
        ts, tn = divmod(int(t_ns[i]), 1_000_000_000)
        ts += day_start
        best_ask, best_bid = asks.keys()[0], bids.keys()[-1]
        thin_a, thin_b = len(asks) < 8, len(bids) < 8
        r = u[i]
        if r < 0.48 or thin_a or thin_b or len(where) < 50:
            side = 1 if thin_b else (-1 if thin_a else int(side_draw[i]))
            if mkt[i] < 0.05:   # marketable limit through the touch
                price = best_ask + int(geo[i]) * tick if side == 1 else best_bid - int(geo[i]) * tick
            elif side == 1:
                price = best_ask - tick * (1 + int(geo[i]))
            else:
                price = best_bid + tick * (1 + int(geo[i]))
            qty = int(lqty[i])
            # the full-depth book matches a marketable order immediately (LOBSTER would log the
            # executions); the generator keeps only the residual so its own book stays uncrossed
            rest, opp = qty, (asks if side == 1 else bids)
            while rest > 0 and len(opp) and (opp.keys()[0] <= price if side == 1 else opp.keys()[-1] >= price):
                lvl_p = opp.keys()[0] if side == 1 else opp.keys()[-1]
                o, q = opp[lvl_p][0]
                take = min(q, rest)
                remove_qty(o, take)
                rest -= take
            oid = add(side, price, rest) if rest > 0 else next_oid
            if rest <= 0:
                next_oid += 1
            msgs[i] = (1, side, qty, price, oid, oid, ts, tn)
        elif r < 0.60 or r < 0.90:
            oid = picker.pick(pick[i])
            side, price = where[oid]
            q = _qty_of(asks if side == -1 else bids, price, oid)
            if r < 0.60 and q > 1:
                c = int(rng.integers(1, q))
                msgs[i] = (2, side, c, price, oid, oid, ts, tn)
                remove_qty(oid, c)
            else:       # delete (LOBSTER type 3, recoded to 2 by the loader)
                msgs[i] = (2, side, q, price, oid, oid, ts, tn)
                remove_qty(oid, q)
        else:
            side = int(side_draw[i])
            book = bids if side == 1 else asks
            lvl_p = book.keys()[-1] if side == 1 else book.keys()[0]
            oid, q = book[lvl_p][0]
            e = int(rng.integers(1, q + 1))
            msgs[i] = (4, side, e, lvl_p, oid, oid, ts, tn)
            remove_qty(oid, e)
    return LobsterDay(msgs=msgs.astype(np.int32), books=books.astype(np.int32), snap_idx=snap_idx, tick_size=tick)


class _LivePicker:
    """Uniform pick over live order ids from a periodically refreshed key list."""

    def __init__(self, where, rng):
        self.where, self.rng, self.keys, self.stale = where, rng, None, 0

    def pick(self, u):
        if self.keys is None or self.stale > 256:
            self.keys, self.stale = list(self.where.keys()), 0
        for _ in range(64):
            oid = self.keys[int(u * len(self.keys)) % len(self.keys)]
            if oid in self.where:
                self.stale += 1
                return oid
            u = self.rng.random()
        self.keys, self.stale = list(self.where.keys()), 0
        return self.keys[int(u * len(self.keys)) % len(self.keys)]


def _qty_of(book, price, oid):
    for o, q in book[price]:
        if o == oid:
            return q
    raise KeyError(oid)
