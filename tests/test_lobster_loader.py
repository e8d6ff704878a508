"""LOBSTER ingestion (hftlob.data.lobster) — restatement of LoadLOBSTER_resample.

Parity status: the reference loader cannot run here (lobster_loader.py imports jax at
module top; no LOBSTER data ships with it), so it is pinned by a hand-made raw day
(tests/golden/lobster_tiny) whose expected post-load arrays are derived line by line
from lobster_loader.py:891-1132, plus structural properties on a generated raw day.
"""
import os
import shutil

import numpy as np
import pandas as pd
import pytest

from hftlob.data import lobster as Lb
from hftlob.data.raw_synthetic import write_raw_lobster_day

HERE = os.path.dirname(os.path.abspath(__file__))
TINY = os.path.join(HERE, "golden", "lobster_tiny")

# Expected post-load rows [type, direction, qty, price, trader_id, order_id, time_s, time_ns]
# (derivation: file rows 0 / 12 fall outside [34200, 34300] s, rows 3 (type 5) and 10
# (type 7) are not types 1-4; executions 4 and 5 share (34200, 400000000, -1) and merge
# into row 5 with qty 4 + 2 and the max price (direction -1); row 6 has direction 1 and
# stays; the delete (row 7) becomes type 2; then the first kept message (row 1) is
# dropped by the alignment shift.  ns = int64((t - int64(t)) * 1e9) in float64, so
# 34200.2 -> 199999999 and 34200.6 -> 599999999, as pandas computes it in the reference.)
TINY_MSGS = [
    [1, -1, 7, 10200, 13, 13, 34200, 199999999],
    [4, -1, 6, 10200, 13, 13, 34200, 400000000],
    [4, 1, 1, 10000, 12, 12, 34200, 400000000],
    [2, 1, 4, 10000, 12, 12, 34200, 500000000],
    [2, -1, 1, 10200, 13, 13, 34200, 599999999],
    [1, 1, 9, 9900, 14, 14, 34250, 0],
    [1, -1, 3, 10300, 15, 15, 34300, 999999999],
]
# kept file rows 1,2,5,6,7,8,9,11; book rows iloc[kept][:-1] -> file rows 1,2,5,6,7,8,9
TINY_BOOK_ROWS = [1, 2, 5, 6, 7, 8, 9]


def _book_row(k):
    return [1000 + k, k, 900 + k, k, 1100 + k, k, 800 + k, k]


def _tiny_loader(tmp_path, type_, length, res, D):
    return Lb.LoadLOBSTER_resample(TINY, str(tmp_path), 2, type_, window_length=length, window_resolution=res,
                                   n_data_msg_per_step=D, day_start=34200, day_end=34300, stock="TINY",
                                   time_period="2026_Oct")


def test_tiny_preprocess():
    d = os.path.join(TINY, "rawLOBSTER", "TINY", "2026_Oct")
    mf = [f for f in os.listdir(d) if "message" in f][0]
    bf = [f for f in os.listdir(d) if "orderbook" in f][0]
    m, ob = Lb.pre_process_msg_ob(Lb.read_message_csv(os.path.join(d, mf)), Lb.read_orderbook_csv(os.path.join(d, bf)),
                                  34200, 34300)
    assert m[Lb.OUT_COLUMNS].to_numpy().tolist() == TINY_MSGS
    assert ob.to_numpy().tolist() == [_book_row(k) for k in TINY_BOOK_ROWS]


def test_tiny_fixed_steps_windows_and_cache(tmp_path):
    # D = 2, 2 steps, a start every step: d_end = 7 - 2*2 = 3 -> starts range(0, 3, 2) = [0, 2]
    ld = _tiny_loader(tmp_path, "fixed_steps", 2, 1, 2)
    msgs, s, e, books, mx = ld.run_loading("tiny")
    assert msgs.tolist() == TINY_MSGS
    assert s.tolist() == [0, 2] and e.tolist() == [4, 6] and mx.tolist() == [4, 4]
    assert books.tolist() == [_book_row(1), _book_row(5)]
    cache = os.path.join(str(tmp_path), "saved_npz", "loaded_lobster_LoadLOBSTER_resample_tiny.npz")
    assert os.path.exists(cache)
    again = ld.run_loading("tiny")                        # served from the npz cache
    for a, b in zip((msgs, s, e, books, mx), again):
        assert np.array_equal(a, b)


def test_tiny_fixed_time_windows(tmp_path):
    # starts range(34200, 34301, 50); window [34200, 34260) holds rows 0..5, [34250, 34310) rows 5..6
    ld = _tiny_loader(tmp_path, "fixed_time", 60, 50, 2)
    msgs, s, e, books, mx = ld.run_loading("tiny_t")
    assert s.tolist() == [0, 5] and e.tolist() == [5, 6] and mx.tolist() == [5, 1]
    assert books.tolist() == [_book_row(1), _book_row(8)]


def test_merge_market_orders_unit():
    df = pd.DataFrame({"time": [1.0] * 5, "type": [4, 4, 1, 4, 4], "order_id": [1, 2, 3, 4, 5],
                       "qty": [3, 4, 9, 5, 6], "price": [100, 101, 99, 90, 91], "direction": [1, 1, 1, 1, -1],
                       "time_s": [1, 1, 1, 1, 1], "time_ns": [5, 5, 5, 5, 5]})
    out = Lb.merge_market_orders(df)
    # executions 0, 1, 3 share (1, 5, +1): kept as row 3, qty 12, min price 90; row 4 (direction -1) alone
    assert out.index.tolist() == [2, 3, 4]
    assert out.loc[3, "qty"] == 12 and out.loc[3, "price"] == 90 and out.loc[3, "order_id"] == 4
    assert out.loc[4, "qty"] == 6 and out.loc[4, "price"] == 91


def test_slice_indices_errors():
    with pytest.raises(ValueError):
        Lb.daily_slice_indices("fixed_steps", 0, 10, 1, 0)
    with pytest.raises(ValueError):
        Lb.daily_slice_indices("fixed_time", 0, 5, 10, 100)   # a single start: not enough range
    with pytest.raises(NotImplementedError):
        Lb.daily_slice_indices("other", 0, 5, 1, 1)


@pytest.fixture(scope="module")
def raw_day(tmp_path_factory):
    root = str(tmp_path_factory.mktemp("lobster"))
    mp, bp = write_raw_lobster_day(root, n_events=12_000, seed=3)
    return root, mp, bp


def test_generated_day_properties(raw_day):
    root, mp, bp = raw_day
    raw_m, raw_b = Lb.read_message_csv(mp), Lb.read_orderbook_csv(bp)
    m, ob = Lb.pre_process_msg_ob(raw_m, raw_b, 34200, 57600)
    assert set(np.unique(m["type"])) <= {1, 2, 4}
    assert m["time_s"].between(34200, 57600).all()
    assert (m["trader_id"] == m["order_id"]).all()
    # the shift: book row i is the raw book after the kept message before message i
    t = raw_m[0].to_numpy()
    keep = (t.astype(np.int64) >= 34200) & (t.astype(np.int64) <= 57600) & raw_m[1].isin([1, 2, 3, 4]).to_numpy()
    assert m.shape[0] == ob.shape[0] < keep.sum()        # merges removed rows
    # execution quantity is conserved by the merge
    ex_raw = raw_m[keep & (raw_m[1] == 4).to_numpy()][3].sum()
    ex_out = m[m["type"] == 4]["qty"].sum()
    first = raw_m[keep].iloc[0]
    assert ex_out == ex_raw - (first[3] if first[1] == 4 else 0)
    # no two executions left with the same stamp and direction
    e = m[m["type"] == 4]
    assert not e.duplicated(["time_s", "time_ns", "direction"]).any()


def test_generated_day_windows(raw_day):
    root, _, _ = raw_day
    ld = Lb.LoadLOBSTER_resample(root, root, 10, "fixed_time", window_length=900, window_resolution=600,
                                 n_data_msg_per_step=50, stock="SYN", time_period="2026_Oct")
    msgs, s, e, books, mx = ld.run_loading("ft")
    t = msgs[:, 6].astype(np.float64) + msgs[:, 7] / 1e9
    starts = list(range(34200, 57601, 600))[:-1]
    assert len(s) == len(starts) and (mx == e - s).all()
    for ws, a, b in zip(starts, s, e):
        assert ws <= t[a] < ws + 900 and ws <= t[b] < ws + 900
        assert a == 0 or t[a - 1] < ws + 1e-6
    assert books.shape == (len(s), 40)
    day = Lb.LoadedDay.from_arrays(msgs, s, e, books, mx)
    assert day.msgs.dtype == np.int32 and day.books.dtype == np.int32
    assert (day.books[:, 0] == np.int64(9999999999).astype(np.int32)).sum() == (books[:, 0] == 9999999999).sum()


def test_init_times_fixed_time():
    from hftlob.config import World_EnvironmentConfig
    from hftlob.data.windows import init_times
    w = World_EnvironmentConfig(ep_type="fixed_time", episode_time=900, start_resolution=600)
    ft = np.zeros((40, 2), np.int32)
    it = init_times(ft, w)
    # base_env.py:287-291: (w * 600) % (57600 - 34200 - 900 + 600) + 34200
    assert it[:, 0].tolist() == [(k * 600) % 23100 + 34200 for k in range(40)] and (it[:, 1] == 0).all()
    w2 = World_EnvironmentConfig()
    assert (init_times(ft + 5, w2) == 5).all()
