"""Order-book engine operators (device tensors in, device tensors out).

Mirrors the reference operator API of ``gymnax_exchange/jaxob/
JaxOrderBookArrays.py`` for the batched case the MARL path uses:

* ``scan_through_entire_array_save_bidask(cfg, key, msg_array, book_state,
  N_steps)`` (:791-823) -> ``((asks, bids, trades), (best_asks[-N:],
  best_bids[-N:]))``
* ``scan_through_entire_array(cfg, key, msg_array, book_state)`` (:736-756)

Every array carries a leading env dimension (the reference is vmapped; here
the batch is explicit).  ``key`` (uint32 words, shape (2,) shared by every
env or (E, 2) per env; None = PRNGKey(0)) only matters for cancel modes 2/3,
where message k of env e draws from split(key_e, M)[k] (:753,784,816).
Functional like the reference: inputs are not modified.  ``book_process_`` is
the in-place form.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Tuple

import torch

from . import _lib
from .config import JAXLOB_Configuration
from .layout import pack_lob_cfg


def _lob(cfg: JAXLOB_Configuration, prng_partitionable: bool = True):
    return pack_lob_cfg(cfg, prng_partitionable)


def _keys(key, E: int, device) -> torch.Tensor:
    """The scan key per env as int32 [E, 2] (uint32 bit patterns)."""
    if key is None:
        return torch.zeros((E, 2), dtype=torch.int32, device=device)
    k = torch.as_tensor(key, device=device)
    if k.dtype != torch.int32:
        k = k.to(torch.int64).bitwise_and(0xFFFFFFFF).to(torch.int64)
        k = torch.where(k >= 2**31, k - 2**32, k).to(torch.int32)
    if k.shape == (2,):
        k = k.expand(E, 2)
    if tuple(k.shape) != (E, 2):
        raise ValueError(f"key must have shape (2,) or ({E}, 2), got {tuple(k.shape)}")
    return k.contiguous()


def _batched(x: torch.Tensor, tail: int) -> torch.Tensor:
    return x if x.dim() == tail + 1 else x.unsqueeze(0)


def book_process_(cfg: JAXLOB_Configuration, msgs: torch.Tensor, asks: torch.Tensor, bids: torch.Tensor,
                  trades: torch.Tensor, best_asks: Optional[torch.Tensor] = None,
                  best_bids: Optional[torch.Tensor] = None, stream=None, keys: Optional[torch.Tensor] = None,
                  prng_partitionable: bool = True) -> None:
    """In place: process msgs [E, M, 8] through (asks, bids [E, nO, 6], trades [E, nT, 8]).
    keys: int32 [E, 2] scan keys (required for cancel_mode 2/3)."""
    E, M = msgs.shape[0], msgs.shape[1]
    for t, shp in ((msgs, (E, M, 8)), (asks, (E, cfg.nOrders, 6)), (bids, (E, cfg.nOrders, 6)),
                   (trades, (E, cfg.nTrades, 8))):
        if tuple(t.shape) != shp or t.dtype != torch.int32:
            raise ValueError(f"expected int32 {shp}, got {t.dtype} {tuple(t.shape)}")
    if best_asks is not None and (tuple(best_asks.shape) != (E, M, 2) or tuple(best_bids.shape) != (E, M, 2)):
        raise ValueError("best_asks / best_bids must be int32 [E, M, 2]")
    if keys is not None and (tuple(keys.shape) != (E, 2) or keys.dtype != torch.int32):
        raise ValueError("keys must be int32 [E, 2]")
    L = _lib.lib()
    c = _lob(cfg, prng_partitionable)
    with torch.cuda.device(msgs.device):
        _lib.check(L.hftlob_book_process(C.byref(c), E, M, _lib.ptr(keys), _lib.ptr(msgs), _lib.ptr(asks),
                                         _lib.ptr(bids), _lib.ptr(trades), _lib.ptr(best_asks), _lib.ptr(best_bids),
                                         _lib.stream_ptr(stream, device=msgs.device)))


def scan_through_entire_array_save_bidask(cfg: JAXLOB_Configuration, key, msg_array: torch.Tensor,
                                          book_state: Tuple[torch.Tensor, torch.Tensor, torch.Tensor],
                                          N_steps: Optional[int] = None, prng_partitionable: bool = True):
    single = msg_array.dim() == 2
    msgs = _batched(msg_array, 2).contiguous()
    asks, bids, trades = (_batched(x, 2).clone().contiguous() for x in book_state)
    E, M = msgs.shape[0], msgs.shape[1]
    ba = torch.empty((E, M, 2), dtype=torch.int32, device=msgs.device)
    bb = torch.empty_like(ba)
    book_process_(cfg, msgs, asks, bids, trades, ba, bb, keys=_keys(key, E, msgs.device),
                  prng_partitionable=prng_partitionable)
    n = M if N_steps is None else N_steps
    ba, bb = ba[:, M - n:], bb[:, M - n:]
    if single:
        asks, bids, trades, ba, bb = asks[0], bids[0], trades[0], ba[0], bb[0]
    return (asks, bids, trades), (ba, bb)


def scan_through_entire_array(cfg: JAXLOB_Configuration, key, msg_array: torch.Tensor,
                              book_state: Tuple[torch.Tensor, torch.Tensor, torch.Tensor],
                              prng_partitionable: bool = True):
    single = msg_array.dim() == 2
    msgs = _batched(msg_array, 2).contiguous()
    asks, bids, trades = (_batched(x, 2).clone().contiguous() for x in book_state)
    book_process_(cfg, msgs, asks, bids, trades, keys=_keys(key, msgs.shape[0], msgs.device),
                  prng_partitionable=prng_partitionable)
    if single:
        return asks[0], bids[0], trades[0]
    return asks, bids, trades


def init_orderside(nOrders: int = 100, n_env: Optional[int] = None, device="cuda") -> torch.Tensor:
    """init_orderside — JaxOrderBookArrays.py:987-997 (all -1)."""
    shape = (nOrders, 6) if n_env is None else (n_env, nOrders, 6)
    return torch.full(shape, -1, dtype=torch.int32, device=device)


def init_trades(nTrades: int = 100, n_env: Optional[int] = None, device="cuda") -> torch.Tensor:
    shape = (nTrades, 8) if n_env is None else (n_env, nTrades, 8)
    return torch.full(shape, -1, dtype=torch.int32, device=device)
