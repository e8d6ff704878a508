"""ctypes binding of libhftlob.so (the HIP/gfx950 library behind include/hftlob.h).

There is deliberately no CPU fallback: if the library is missing, or a call
is made without a GPU, this module raises.  The CPU restatement under
``oracle/`` is test infrastructure and is never imported from here.
"""
from __future__ import annotations

import ctypes as C
import os

from .layout import EnvCfg, LobCfg, StepOut


class LaunchInfo(C.Structure):
    """hftlob_launch_info (include/hftlob.h): the kernel instantiation a config launches."""
    _fields_ = [("slot_sets", C.c_int32), ("nfix", C.c_int32), ("random_cancel", C.c_int32),
                ("rows_alias", C.c_int32), ("lds_bytes", C.c_int32), ("tick_magic", C.c_uint32),
                ("key_batch", C.c_int32)]

LIB_PATH = os.environ.get("HFTLOB_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libhftlob.so")
ABI_VERSION = 7
EXPORTS = ("hftlob_version", "hftlob_last_error", "hftlob_book_process", "hftlob_env_reset",
           "hftlob_env_step", "hftlob_env_step_sampled", "hftlob_env_rollout_sampled", "hftlob_rollout_prepare",
           "hftlob_env_lds_bytes", "hftlob_env_launch_info",
           "hftlob_sample_actions", "hftlob_split_keys")

_lib = None


class HftlobError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"hftlob error {code}: {msg}")
        self.code = code


def lib() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is not built; run `python -c 'import __graft_entry__ as g; g.build()'`")
    L = C.CDLL(LIB_PATH)
    vp, i32 = C.c_void_p, C.c_int
    L.hftlob_version.restype = i32
    L.hftlob_last_error.restype = C.c_char_p
    L.hftlob_book_process.argtypes = [C.POINTER(LobCfg), i32, i32, vp, vp, vp, vp, vp, vp, vp, vp]
    L.hftlob_book_process.restype = i32
    L.hftlob_env_reset.argtypes = [C.POINTER(EnvCfg), i32, vp, vp, vp, vp, C.POINTER(StepOut), vp]
    L.hftlob_env_reset.restype = i32
    L.hftlob_env_step.argtypes = [C.POINTER(EnvCfg), i32, vp, vp, vp, vp, vp, C.POINTER(StepOut), vp]
    L.hftlob_env_step.restype = i32
    L.hftlob_env_step_sampled.argtypes = [C.POINTER(EnvCfg), i32, vp, vp, vp, vp, vp, vp, C.POINTER(StepOut), vp]
    L.hftlob_env_step_sampled.restype = i32
    L.hftlob_env_rollout_sampled.argtypes = [C.POINTER(EnvCfg), i32, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp,
                                             C.POINTER(StepOut), i32, i32, vp]
    L.hftlob_env_rollout_sampled.restype = i32
    L.hftlob_rollout_prepare.argtypes = [i32, vp]
    L.hftlob_rollout_prepare.restype = i32
    L.hftlob_env_lds_bytes.argtypes = [C.POINTER(EnvCfg)]
    L.hftlob_env_lds_bytes.restype = i32
    L.hftlob_env_launch_info.argtypes = [C.POINTER(EnvCfg), C.POINTER(LaunchInfo)]
    L.hftlob_env_launch_info.restype = i32
    L.hftlob_sample_actions.argtypes = [C.POINTER(EnvCfg), i32, vp, vp, vp]
    L.hftlob_sample_actions.restype = i32
    L.hftlob_split_keys.argtypes = [i32, i32, i32, vp, vp, vp]
    L.hftlob_split_keys.restype = i32
    if L.hftlob_version() != ABI_VERSION:
        raise RuntimeError(f"libhftlob ABI {L.hftlob_version()} != {ABI_VERSION}")
    _lib = L
    return L


def check(rc: int) -> None:
    if rc != 0:
        raise HftlobError(rc, lib().hftlob_last_error().decode())


def ptr(t) -> int:
    """Device pointer of a CUDA (HIP) tensor; refuses host tensors loudly."""
    if t is None:
        return None
    if not t.is_cuda:
        raise RuntimeError("hftlob kernels need device (HIP) tensors; got a CPU tensor")
    if not t.is_contiguous():
        raise RuntimeError("hftlob kernels need contiguous tensors")
    return t.data_ptr()


def stream_ptr(stream=None, device=None) -> int:
    """hipStream_t of `stream`, else of torch's current stream on `device` (default: the
    current device)."""
    import torch
    s = stream if stream is not None else torch.cuda.current_stream(device)
    return s.cuda_stream
