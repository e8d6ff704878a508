"""LOBSTER ingestion: raw ``*_message_*.csv`` / ``*_orderbook_*.csv`` day pairs
to the post-load arrays the env replays (host, once per dataset).

Restates ``LoadLOBSTER_resample`` (``gymnax_exchange/jaxlobster/lobster_loader.py:516-1071``)
and ``merge_market_orders`` (``:1073-1132``):

* ``pre_process_msg_ob`` (``:891-945``): time split into (s, ns) int64
  (``ns = int64((t - int64(t)) * 1e9)``, float64 as pandas does), drop rows
  outside ``[day_start, day_end]`` seconds, keep types 1-4, merge same-stamp
  executions, recode type 3 (delete) -> 2 (cancel), ``trader_id = order_id``,
  then the one-row alignment shift: book row i is the state BEFORE message i.
* ``daily_slice_indices`` / ``get_inits_day`` (``:971-1071``): window starts
  every ``D * window_resolution`` messages (``fixed_steps``) or every
  ``window_resolution`` seconds (``fixed_time``, first/last message index
  inside ``[start, start + window_length)``, empty windows skipped), the L2
  snapshot at each start, the int message rows
  ``[type, direction, qty, price, trader_id, order_id, time_s, time_ns]``.
* ``LoadLOBSTER_resample.run_loading`` (``:626-695``): day files in sorted
  order, per-day window indices offset by the messages of earlier days,
  concatenated; cached as ``saved_npz/loaded_lobster_LoadLOBSTER_resample_<suffix>.npz``
  under ``alphatradePath`` (our own cache: read back with ``allow_pickle=False``).

The arrays stay int64 here; ``LoadedDay`` converts them to the int32 the env
uses (JAX with x64 disabled wraps int64 -> int32 the same way, e.g. the empty
level price 9999999999 -> 1410065407).
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from glob import glob
from typing import List, Optional, Sequence, Tuple

import numpy as np
import pandas as pd

MSG_COLUMNS = ["time", "type", "order_id", "qty", "price", "direction", "time_s", "time_ns"]
OUT_COLUMNS = ["type", "direction", "qty", "price", "trader_id", "order_id", "time_s", "time_ns"]


# ----------------------------------------------------------------- parsing
def read_message_csv(path: str) -> pd.DataFrame:
    """The first 6 columns of a LOBSTER message file, header-less (time float, ints)."""
    return pd.read_csv(path, usecols=range(6), header=None, engine="c", na_filter=False)


def read_orderbook_csv(path: str) -> pd.DataFrame:
    return pd.read_csv(path, header=None, engine="c", na_filter=False)


# ------------------------------------------------------------ preprocessing
def merge_market_orders(msg: pd.DataFrame) -> pd.DataFrame:
    """lobster_loader.py:1073-1132.  Executions (type 4) sharing (time_s, time_ns,
    direction) collapse into the group's LAST row (by position): qty = group sum,
    price = group max for direction -1, min otherwise.  Other rows untouched;
    index labels are kept (the caller aligns the book rows by them)."""
    ex = msg["type"].to_numpy() == 4
    if not ex.any():
        return msg.copy()
    out = msg.copy()
    e = out.loc[ex, ["time_s", "time_ns", "direction", "qty", "price"]]
    keys = [e["time_s"], e["time_ns"], e["direction"]]
    g = e.groupby(keys, sort=False)
    qty = g["qty"].transform("sum")
    pmax = g["price"].transform("max")
    pmin = g["price"].transform("min")
    is_last = g.cumcount(ascending=False).to_numpy() == 0
    size = g["qty"].transform("size").to_numpy()
    merged = size > 1
    upd = e.index[is_last & merged]
    out.loc[upd, "qty"] = qty.loc[upd].to_numpy()
    out.loc[upd, "price"] = np.where(e.loc[upd, "direction"].to_numpy() == -1, pmax.loc[upd].to_numpy(),
                                     pmin.loc[upd].to_numpy())
    return out.drop(index=e.index[~is_last])


def pre_process_msg_ob(message_day: pd.DataFrame, orderbook_day: pd.DataFrame, day_start: int,
                       day_end: int) -> Tuple[pd.DataFrame, pd.DataFrame]:
    """lobster_loader.py:891-945 (LoadLOBSTER_resample._pre_process_msg_ob)."""
    m = message_day.copy()
    t = m[0].to_numpy(dtype=np.float64)
    ts = t.astype(np.int64)                                  # truncation, as Series.astype(int64)
    m[6] = ts
    m[7] = ((t - ts) * 1_000_000_000).astype(np.int64)
    m = m[(m[6] >= day_start) & (m[6] <= day_end)]
    m.columns = MSG_COLUMNS
    m = m[m["type"].isin([1, 2, 3, 4])].copy()
    m = merge_market_orders(m)
    valid = m.index.to_numpy()
    m = m.reset_index(drop=True)
    m.loc[m["type"] == 3, "type"] = 2
    m["trader_id"] = m["order_id"]
    ob = orderbook_day.iloc[valid, :].reset_index(drop=True)
    ob = ob.iloc[:-1, :].reset_index(drop=True)
    m = m.iloc[1:, :].reset_index(drop=True)
    if m.shape[0] != ob.shape[0]:
        raise ValueError("Orderbook and message dataframe mismatch after pre-processing")
    return m, ob


def daily_slice_indices(window_type: str, start: int, end: int, interval: int, n_data_msg_per_step: int) -> List[int]:
    """lobster_loader.py:971-1002 (_daily_slice_indeces): candidate window starts."""
    D = n_data_msg_per_step
    if window_type == "fixed_steps":
        if D == 0:
            raise ValueError("n_data_msg_per_step cannot be 0 if using 'fixed_steps' as an episode end condition.")
        if D < 0:
            raise ValueError("Negative messages per step makes no sense...")
        end_index = (end - start) // D * D + start + 1
        idx = list(range(start, end_index, D * interval))
    elif window_type == "fixed_time":
        idx = list(range(start, end + 1, interval))
    else:
        raise NotImplementedError('Use either "fixed_time" or "fixed_steps"')
    if len(idx) < 2:
        raise ValueError("Not enough range to get a slice")
    return idx


def get_inits_day(m: pd.DataFrame, ob: pd.DataFrame, window_type: str, window_length: int,
                  window_resolution: int, n_data_msg_per_step: int, day_start: int, day_end: int):
    """lobster_loader.py:1004-1071 (_get_inits_day) -> (msgs int64 (N,8), index_s, index_e, init_OBs)."""
    D = n_data_msg_per_step
    if window_type == "fixed_time":
        d_start, d_end = day_start, day_end
    else:
        d_start, d_end = 0, m.shape[0] - window_length * D
    idx = daily_slice_indices(window_type, d_start, d_end, window_resolution, D)
    if window_type == "fixed_steps":
        index_s = np.asarray(idx, dtype=np.int64)
        index_e = index_s + D * window_length
    else:
        t = m["time"].to_numpy(dtype=np.float64)
        s_list, e_list = [], []
        for ws in idx[:-1]:
            inside = np.flatnonzero((t >= ws) & (t < ws + window_length))
            if inside.size:                       # empty windows are skipped (reference prints a warning)
                s_list.append(int(inside[0]))
                e_list.append(int(inside[-1]))
        index_s = np.asarray(s_list, dtype=np.int64)
        index_e = np.asarray(e_list, dtype=np.int64)
    init_obs = ob.to_numpy(dtype=np.int64)[index_s] if index_s.size else np.zeros((0, ob.shape[1]), np.int64)
    msgs = m[OUT_COLUMNS].to_numpy(dtype=np.int64)
    return msgs, index_s, index_e, init_obs


def load_day(message_file: str, orderbook_file: str, window_type: str, window_length: int, window_resolution: int,
             n_data_msg_per_step: int, day_start: int, day_end: int):
    """One file pair -> (msgs, starts, ends, books, max_msgs) in day-local indices (read_pair, :758-831)."""
    mb = os.path.basename(message_file).replace("_message_", "_PLACEHOLDER_").replace(".csv", "")
    bb = os.path.basename(orderbook_file).replace("_orderbook_", "_PLACEHOLDER_").replace(".csv", "")
    if mb != bb:
        raise ValueError(f"Message and orderbook file mismatch: {message_file} vs {orderbook_file}")
    m, ob = pre_process_msg_ob(read_message_csv(message_file), read_orderbook_csv(orderbook_file), day_start, day_end)
    msgs, s, e, books = get_inits_day(m, ob, window_type, window_length, window_resolution, n_data_msg_per_step,
                                      day_start, day_end)
    return msgs, s, e, books, e - s


# ------------------------------------------------------------------ loader
class LoadLOBSTER_resample:
    """lobster_loader.py:516-625: same constructor, same file discovery
    (``<datapath>/rawLOBSTER/<stock>/<period>/*message*.csv`` / ``*orderbook*.csv``,
    comma-separated stock / period lists), ``run_loading`` returning
    ``(msgs, starts, ends, books, max_msgs_in_windows_arr)``."""

    def __init__(self, datapath, atpath, n_Levels=10, type_="fixed_time", window_length=1800, window_resolution=60,
                 n_data_msg_per_step=100, day_start=34200, day_end=57600, stock="AMZN",
                 time_period="2017Jan_oneday"):
        stocks = [s.strip() for s in stock.split(",")] if isinstance(stock, str) else list(stock)
        periods = [p.strip() for p in time_period.split(",")] if isinstance(time_period, str) else list(time_period)
        self.stock, self.time_period = stock, time_period
        self.datapaths = [f"{datapath}/rawLOBSTER/{s}/{p}/" for s in stocks for p in periods]
        self.window_type, self.window_length, self.window_resolution = type_, window_length, window_resolution
        self.n_data_msg_per_step, self.day_start, self.day_end = n_data_msg_per_step, day_start, day_end
        self.n_Levels, self.alphatrade_path = n_Levels, atpath
        mf, bf = [], []
        for d in self.datapaths:
            mf += [f for f in glob(d + "*message*.csv") if os.path.getsize(f) > 0]
            bf += [f for f in glob(d + "*orderbook*.csv") if os.path.getsize(f) > 0]
        self.message_files, self.book_files = sorted(mf), sorted(bf)

    def _get_save_filename(self, string_suffix="NONE_GIVEN") -> str:
        os.makedirs(os.path.join(self.alphatrade_path, "saved_npz"), exist_ok=True)
        return os.path.join(self.alphatrade_path, f"saved_npz/loaded_lobster_{type(self).__name__}_{string_suffix}.npz")

    def _load_files(self):
        if not self.message_files:
            raise FileNotFoundError(f"No data files found in {self.datapaths}. Check that dataPath, stock, and "
                                    "timePeriod are correct in your env config.")
        if len(self.message_files) != len(self.book_files):
            raise ValueError("message / orderbook file counts differ")
        out = []
        for mf, bf in zip(self.message_files, self.book_files):
            out.append(load_day(mf, bf, self.window_type, self.window_length, self.window_resolution,
                                self.n_data_msg_per_step, self.day_start, self.day_end))
        return out

    def run_loading(self, filename_suffix="NONE_GIVEN"):
        path = self._get_save_filename(filename_suffix)
        if os.path.exists(path):
            with np.load(path, allow_pickle=False) as z:
                return (z["msgs"], z["starts"], z["ends"], z["obs"], z["max_msgs_in_windows_arr"])
        days = self._load_files()
        msgs, starts, ends, obs, mx = [], [], [], [], []
        off = 0
        for m, s, e, b, n in days:
            msgs.append(m)
            starts.append(s + off)
            ends.append(e + off)
            obs.append(b)
            mx.append(n)
            off += m.shape[0]
        msgs, starts, ends = np.concatenate(msgs, 0), np.concatenate(starts, 0), np.concatenate(ends, 0)
        obs, mx = np.concatenate(obs, 0), np.concatenate(mx, 0)
        np.savez_compressed(path, msgs=msgs, starts=starts, ends=ends, obs=obs, max_msgs_in_windows_arr=mx)
        return msgs, starts, ends, obs, mx


def filename_suffix(w) -> str:
    """BaseLOBEnv._get_filename_suffix (base_env.py:398-411)."""
    return "_".join(str(x) for x in (w.stock, w.timePeriod, w.book_depth, w.ep_type, w.episode_time,
                                     w.start_resolution, w.n_data_msg_per_step, w.day_start, w.day_end))


@dataclass
class LoadedDay:
    """Post-load arrays as the env consumes them (int32, JAX x64-disabled wrap)."""
    msgs: np.ndarray          # (N, 8) int32
    starts: np.ndarray        # (W,) int32
    ends: np.ndarray          # (W,) int32
    books: np.ndarray         # (W, 4*depth) int32
    max_msgs: np.ndarray      # (W,) int32

    @classmethod
    def from_arrays(cls, msgs, starts, ends, books, max_msgs) -> "LoadedDay":
        w = lambda a: np.asarray(a, dtype=np.int64).astype(np.int32)  # noqa: E731  (int64 -> int32 wrap)
        return cls(msgs=np.ascontiguousarray(w(msgs)), starts=w(starts), ends=w(ends), books=w(books),
                   max_msgs=w(max_msgs))


def load_from_config(world_cfg, alphatrade_path: Optional[str] = None) -> LoadedDay:
    """BaseLOBEnv.__init__'s loading (base_env.py:157-176) for a World_EnvironmentConfig."""
    w = world_cfg
    loader = LoadLOBSTER_resample(w.dataPath, alphatrade_path or w.alphatradePath, w.book_depth, w.ep_type,
                                  window_length=w.episode_time, n_data_msg_per_step=w.n_data_msg_per_step,
                                  window_resolution=w.start_resolution, day_start=w.day_start, day_end=w.day_end,
                                  stock=w.stock, time_period=w.timePeriod)
    return LoadedDay.from_arrays(*loader.run_loading(filename_suffix(w)))


def raw_day_files(datapath: str, stock: str, period: str) -> Sequence[str]:
    return sorted(glob(f"{datapath}/rawLOBSTER/{stock}/{period}/*.csv"))
