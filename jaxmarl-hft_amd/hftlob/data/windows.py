"""Episode windows and initial-book messages (host, once per dataset).

* ``fixed_steps_windows`` restates ``LoadLOBSTER_resample._daily_slice_indeces``
  + ``_get_inits_day`` for ``ep_type="fixed_steps"``
  (``jaxlobster/lobster_loader.py:956-1071``): windows start every
  ``n_data_msg_per_step * start_resolution`` messages, each holds
  ``n_data_msg_per_step * episode_time`` messages.
* ``init_messages`` restates ``BaseLOBEnv._get_state_from_data.get_initial_orders``
  (``jaxen/base_env.py:245-273``): the 10-level L2 snapshot becomes 20 limit
  messages ``[1, -1/+1, q, p, oid=init_id, tid=init_id-k, t, ns]`` (asks on even
  rows) stamped with the window's first message time.
* ``loaded_rows`` assembles the LoadedEnvState fields (init_time, window_index,
  max_steps_in_episode = max_msgs // D + 1, start_index, step_counter = 0;
  ``base_env.py:285-296, 320-326``) around the processed init books.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


@dataclass
class Windows:
    starts: np.ndarray        # (W,) start message index
    ends: np.ndarray          # (W,)
    max_msgs: np.ndarray      # (W,) messages per window
    books: np.ndarray         # (W, 4*depth) L2 snapshot before each start


def fixed_steps_windows(n_msgs: int, n_data_msg_per_step: int, episode_time: int, start_resolution: int) -> np.ndarray:
    D = n_data_msg_per_step
    if D <= 0:
        raise ValueError("n_data_msg_per_step must be positive for 'fixed_steps'")
    d_end = n_msgs - episode_time * D
    end_index = (d_end - 0) // D * D + 0 + 1
    starts = np.arange(0, end_index, D * start_resolution, dtype=np.int64)
    if len(starts) < 2:
        raise ValueError("Not enough range to get a slice")
    return starts


def make_windows(day, world_cfg) -> Windows:
    """Window table for a generated day (``day.books`` at ``day.snap_idx``, fixed_steps) or a
    ``LoadedDay`` from the LOBSTER loader (its own starts / ends / books, either episode type)."""
    if hasattr(day, "starts"):                      # hftlob.data.lobster.LoadedDay
        return Windows(starts=day.starts.astype(np.int32), ends=day.ends.astype(np.int32),
                       max_msgs=day.max_msgs.astype(np.int32), books=day.books.astype(np.int32))
    if world_cfg.ep_type != "fixed_steps":
        raise ValueError("synthetic LobsterDay windows are fixed_steps; load fixed_time windows with "
                         "hftlob.data.lobster (LoadLOBSTER_resample)")
    D = world_cfg.n_data_msg_per_step
    starts = fixed_steps_windows(day.msgs.shape[0], D, world_cfg.episode_time, world_cfg.start_resolution)
    snap_of = {int(s): k for k, s in enumerate(day.snap_idx)}
    missing = [int(s) for s in starts if int(s) not in snap_of]
    if missing:
        raise ValueError(f"no L2 snapshot at window starts {missing[:4]}...; generate with snap_every = D*start_resolution")
    books = np.stack([day.books[snap_of[int(s)]] for s in starts]).astype(np.int32)
    n = D * world_cfg.episode_time
    return Windows(starts=starts.astype(np.int32), ends=(starts + n).astype(np.int32),
                   max_msgs=np.full(len(starts), n, dtype=np.int32), books=books)


def init_messages(books: np.ndarray, first_times: np.ndarray, depth: int, init_id: int) -> np.ndarray:
    """(W, 2*depth, 8) int32 init limit messages, one block per window."""
    W = books.shape[0]
    data = books.reshape(W, 2 * depth, 2).astype(np.int32)
    m = np.zeros((W, 2 * depth, 8), dtype=np.int32)
    m[:, :, 3] = data[:, :, 0]
    m[:, :, 2] = data[:, :, 1]
    m[:, :, 0] = 1
    m[:, 0::2, 1] = -1
    m[:, 1::2, 1] = 1
    m[:, :, 4] = init_id
    m[:, :, 5] = init_id - np.arange(2 * depth, dtype=np.int32)[None, :]
    m[:, :, 6] = first_times[:, None, 0]
    m[:, :, 7] = first_times[:, None, 1]
    return m


def init_times(first_times: np.ndarray, world_cfg) -> np.ndarray:
    """LoadedEnvState.init_time (base_env.py:287-291): the window's first message time for
    fixed_steps; for fixed_time ``[(w * res) % (day_end - day_start - episode_time + res) + day_start, 0]``."""
    w = world_cfg
    if getattr(w, "ep_type", "fixed_steps") != "fixed_time":
        return first_times.astype(np.int32)
    W = first_times.shape[0]
    res = w.start_resolution
    t0 = (np.arange(W, dtype=np.int64) * res) % (w.day_end - w.day_start - w.episode_time + res) + w.day_start
    return np.stack([t0, np.zeros(W, np.int64)], 1).astype(np.int32)


def loaded_rows(asks: np.ndarray, bids: np.ndarray, trades: np.ndarray, first_times: np.ndarray, win: Windows,
                n_data_msg_per_step: int, init_rec_words: int, world_cfg=None) -> np.ndarray:
    """(W, init_rec_words) int32 LoadedEnvState rows in the record layout."""
    W, nO = asks.shape[0], asks.shape[1]
    nT = trades.shape[1]
    rows = np.zeros((W, init_rec_words), dtype=np.int32)
    rows[:, 0:6 * nO] = asks.reshape(W, -1)
    rows[:, 6 * nO:12 * nO] = bids.reshape(W, -1)
    rows[:, 12 * nO:12 * nO + 8 * nT] = trades.reshape(W, -1)
    o = 12 * nO + 8 * nT
    it = init_times(first_times, world_cfg) if world_cfg is not None else first_times
    rows[:, o + 0] = it[:, 0]
    rows[:, o + 1] = it[:, 1]
    rows[:, o + 2] = np.arange(W)
    rows[:, o + 3] = win.max_msgs // n_data_msg_per_step + 1
    rows[:, o + 4] = win.starts
    rows[:, o + 5] = 0
    return rows
