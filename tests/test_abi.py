"""The C-ABI library without a GPU: it loads, exports every entry point that
include/hftlob.h declares, agrees with the host's ctypes structs on sizes and
offsets, and rejects bad calls with the documented codes before any device
work (hftlob.h: HFTLOB_ENULL / EINVAL / ESHAPE)."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from hftlob import _lib
from hftlob.config_io import builtin_config
from hftlob.layout import AgentTypeCfg, EnvCfg, LobCfg, StepOut, pack_env_cfg, pack_lob_cfg
from oracle import pyoracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "hftlob.h")


def _declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"\b(hftlob_[a-z_]+)\s*\(", src)))


def test_header_declares_the_exports():
    assert _declared() == sorted(_lib.EXPORTS)


def test_library_exports_every_declared_symbol():
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libhftlob.so not built (run __graft_entry__.build())")
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    syms = {ln.split()[-1] for ln in out.splitlines() if ln.strip()}
    missing = [s for s in _declared() if s not in syms]
    assert not missing, missing
    L = _lib.lib()                                   # loads, checks the ABI version
    assert L.hftlob_version() == _lib.ABI_VERSION


def test_struct_layout_matches_c():
    lay = O.abi_layout()
    assert lay[0] == C.sizeof(LobCfg)
    assert lay[1] == C.sizeof(AgentTypeCfg)
    assert lay[2] == C.sizeof(EnvCfg)
    assert lay[3] == EnvCfg.types.offset
    assert lay[4] == AgentTypeCfg.rebate_factor.offset
    assert lay[5] == C.sizeof(StepOut)
    assert lay[6] == EnvCfg.info_words.offset
    assert lay[7] == AgentTypeCfg.task.offset


@pytest.fixture(scope="module")
def L():
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libhftlob.so not built")
    return _lib.lib()


def _env_cfg(name="2_player_fq_fqc"):
    c, _ = pack_env_cfg(builtin_config(name), 10, 100_000, True)
    return c


def test_error_null_and_shape(L):
    assert L.hftlob_book_process(None, 1, 1, None, None, None, None, None, None, None, None) == -2
    lob = pack_lob_cfg(builtin_config("2_player_fq_fqc").world_config)
    assert L.hftlob_book_process(C.byref(lob), -1, 1, None, None, None, None, None, None, None, None) == -3
    assert L.hftlob_book_process(C.byref(lob), 0, 1, None, None, None, None, None, None, None, None) == 0  # empty batch
    assert L.hftlob_book_process(C.byref(lob), 4, 8, None, None, None, None, None, None, None, None) == -2
    assert b"null" in L.hftlob_last_error()
    c = _env_cfg()
    out = StepOut()
    assert L.hftlob_env_step(C.byref(c), 4, None, None, None, None, None, C.byref(out), None) == -2
    assert L.hftlob_env_reset(None, 4, None, None, None, None, None, None) == -2
    assert L.hftlob_split_keys(4, 0, 1, None, None, None) == -3
    k = C.c_void_p(64)
    assert L.hftlob_env_step_sampled(C.byref(c), 4, k, None, None, k, k, k, C.byref(out), None) == -2
    assert L.hftlob_env_step_sampled(C.byref(c), 4, k, k, None, k, k, k, C.byref(out), None) == -1  # key_in == key_out
    assert L.hftlob_sample_actions(None, 4, None, None, None) == -2
    # hftlob_env_rollout_sampled(cfg, n_env, key_e0, key_n, n_steps, key_in, key_out, key_scratch, actions,
    #   msgs, init, state, out, per_step, n_slices, stream): argument checks run before any HIP call
    R = L.hftlob_env_rollout_sampled
    assert R(None, 4, 0, 4, 8, k, k, k, None, k, k, k, C.byref(out), 0, 2, None) == -2           # null cfg
    assert R(C.byref(c), -1, 0, 4, 8, k, k, k, None, k, k, k, C.byref(out), 0, 2, None) == -3    # negative n_env
    assert R(C.byref(c), 4, 0, 4, -1, k, k, k, None, k, k, k, C.byref(out), 0, 2, None) == -3    # negative n_steps
    assert R(C.byref(c), 4, 2, 5, 8, k, k, k, None, k, k, k, C.byref(out), 0, 2, None) == -3     # key_e0 + n_env > key_n
    assert R(C.byref(c), 4, -1, 8, 8, k, k, k, None, k, k, k, C.byref(out), 0, 2, None) == -3    # negative key_e0
    assert R(C.byref(c), 4, 0, 4, 8, k, k, k, None, k, k, k, C.byref(out), 0, -1, None) == -1    # n_slices < 0
    assert R(C.byref(c), 4, 0, 4, 8, k, k, k, None, k, k, k, C.byref(out), 0, 5, None) == -1     # n_slices > 4
    assert R(C.byref(c), 0, 0, 4, 8, k, k, k, None, k, k, k, C.byref(out), 0, 2, None) == 0      # empty batch
    assert R(C.byref(c), 4, 0, 4, 0, k, k, k, None, k, k, k, C.byref(out), 0, 2, None) == 0      # no steps
    assert R(C.byref(c), 4, 0, 4, 8, k, None, k, None, k, k, k, C.byref(out), 0, 2, None) == -2  # null key_out
    assert R(C.byref(c), 4, 0, 4, 8, k, k, k, None, k, k, k, C.byref(out), 0, 2, None) == -2     # null outputs
    full = StepOut(k, k, k, k, None)
    k2 = C.c_void_p(128)
    assert R(C.byref(c), 4, 0, 4, 8, k, k2, None, None, k, k, k, C.byref(full), 0, 2, None) == -2  # null scratch
    assert R(C.byref(c), 4, 0, 4, 8, k, k, k, None, k, k, k, C.byref(full), 0, 2, None) == -1    # key_in == key_out
    assert L.hftlob_rollout_prepare(-1, None) == -1
    assert L.hftlob_rollout_prepare(5, None) == -1


@pytest.mark.parametrize("field,value,code", [("cancel_mode", 4, -1), ("type_4_interpretation", 3, -1),
                                              ("n_orders", 0, -3), ("n_trades", 257, -3)])
def test_error_bad_lob_cfg(L, field, value, code):
    lob = pack_lob_cfg(builtin_config("2_player_fq_fqc").world_config)
    setattr(lob, field, value)
    dummy = C.c_void_p(16)  # never dereferenced: validation fails first
    assert L.hftlob_book_process(C.byref(lob), 1, 1, dummy, dummy, dummy, dummy, dummy, None, None, None) == code


def test_random_cancel_needs_keys(L):
    lob = pack_lob_cfg(builtin_config("2_player_fq_fqc").world_config)
    lob.cancel_mode = 2
    dummy = C.c_void_p(16)  # never dereferenced: the NULL keys are refused first
    assert L.hftlob_book_process(C.byref(lob), 1, 1, None, dummy, dummy, dummy, dummy, None, None, None) == -2
    assert b"keys" in L.hftlob_last_error()


def test_error_bad_env_cfg(L):
    dummy = C.c_void_p(16)
    out = StepOut(16, 16, 16, 16, None)
    for mutate, code in ((lambda c: setattr(c, "ep_type", 2), -1),
                         (lambda c: setattr(c, "n_agents", 3), -1),
                         (lambda c: setattr(c, "n_msgs", 1000), -3),
                         (lambda c: setattr(c, "tick_size", 0), -1),      # tick_floordiv needs a tick >= 1
                         (lambda c: setattr(c.types[0], "kind", 7), -1),
                         (lambda c: setattr(c, "action_words", 3), -1),
                         (lambda c: setattr(c.types[0], "action_width", 2), -1),
                         (lambda c: setattr(c.types[1], "action_space", 4), -1),     # fixed_prices, width 1 != 13
                         (lambda c: setattr(c.types[1], "action_space", 5), -1)):
        c = _env_cfg()
        mutate(c)
        rc = L.hftlob_env_step(C.byref(c), 1, dummy, dummy, dummy, dummy, dummy, C.byref(out), None)
        assert rc == code, (rc, code)


def test_device_tensors_required():
    import torch
    with pytest.raises(RuntimeError, match="device"):
        _lib.ptr(torch.zeros(4, dtype=torch.int32))


@pytest.mark.parametrize("name,agents,part,kb", [("2_player_fq_fqc", None, True, True),
                                                 ("2_player_fq_fqc", None, False, False),
                                                 ("3_player_fq_fqc_dir", None, True, False),
                                                 ("default", [1, 1], True, True),
                                                 ("default", [5, 5], True, False),
                                                 ("default", [10, 10], True, False)])
def test_env_lds_bytes(L, name, agents, part, kb):
    """hftlob_env_lds_bytes (the LDS the step / rollout launches reserve per env, which
    MARLEnv.resident_envs sizes launch shapes from) on both sides of the rollout's key-batch rule
    (kb_ok: partitionable keys, <= 3 agents, <= 8 action rows, 6 + agents + rows <= 16):
    [rows (C+A)*8][action extras][asks 6 nO][bids 6 nO][trades 8 nT][pad 64*4][key batches 4 x row], the
    rows inside the trade log for Speed_test's [5,5] and [10,10] (16 envs per CU instead of 14 / 11)."""
    import dataclasses
    cfg = builtin_config(name)
    if agents:
        cfg = dataclasses.replace(cfg, number_of_agents_per_type=agents)
    c, _ = pack_env_cfg(cfg, 4, 1000, part)
    ok = (part and c.n_agents <= 3 and c.n_action_msgs <= 8 and c.n_types <= 6
          and 6 + c.n_agents + c.n_action_msgs <= 16)
    assert ok == kb
    ar = c.n_cancel_msgs + c.n_action_msgs
    rest = 4 * (((c.n_agents * 6 + 3) & ~3) + 12 * c.lob.n_orders + 8 * c.lob.n_trades + 64 * 4
                + (4 * (6 + c.n_agents + c.n_action_msgs) if kb else 0))
    # the agent rows live in the trade log (lds_map, use_rows_alias) only in the 100/100 kernel, when
    # they fit and their own region would hold the env above 160 KB / 16
    # (rows_in_trades: at most two message chunks of rows, ending before the pad's scratch row)
    alias = (c.lob.n_orders == c.lob.n_trades == 100 and c.lob.cancel_mode < 2 and ar <= 128
             and 8 * ar <= 8 * c.lob.n_trades + 192 and rest + 4 * ar * 8 > 160 * 1024 // 16)
    assert alias == (agents in ([5, 5], [10, 10]))
    assert L.hftlob_env_lds_bytes(C.byref(c)) == rest + (0 if alias else 4 * ar * 8)
    info = _lib.LaunchInfo()
    assert L.hftlob_env_launch_info(C.byref(c), C.byref(info)) == 0
    assert (info.slot_sets, info.nfix, info.random_cancel, info.rows_alias) == (2, 100, 0, int(alias))
    assert info.lds_bytes == L.hftlob_env_lds_bytes(C.byref(c))
    assert info.key_batch == int(kb)
    c.ep_type = 2
    assert L.hftlob_env_lds_bytes(C.byref(c)) == -1   # an invalid cfg: its error code
    assert L.hftlob_env_launch_info(C.byref(c), C.byref(info)) == -1


def tick_magic(d: int) -> int:
    """ceil(2^(31+l) / d), l = ceil(log2 d): the multiplier of tick_floordiv (tools/magic_check.c)"""
    l = (d - 1).bit_length() if d > 1 else 0
    return -(-(1 << (31 + l)) // d)


@pytest.mark.parametrize("tick", [1, 2, 3, 7, 25, 100, 128, 1000, 12345, 2 ** 24 + 1, 2 ** 31 - 1])
def test_launch_info_tick_magic(L, tick):
    """the library derives tick_magic from tick_size for every launch (a caller's value is ignored);
    the multiplier is < 2^32 and makes (n * m) >> (31 + l) == n // d on sampled int32 numerators"""
    import dataclasses
    import numpy as np
    cfg = builtin_config("2_player_fq_fqc")
    cfg = dataclasses.replace(cfg, world_config=dataclasses.replace(cfg.world_config, tick_size=tick))
    c, _ = pack_env_cfg(cfg, 4, 1000, True)
    c.tick_magic = 12345  # ignored
    info = _lib.LaunchInfo()
    assert L.hftlob_env_launch_info(C.byref(c), C.byref(info)) == 0
    m = tick_magic(tick)
    assert info.tick_magic == m < 2 ** 32
    l = (tick - 1).bit_length() if tick > 1 else 0
    n = np.concatenate([np.arange(0, 5000), np.random.default_rng(tick).integers(0, 2 ** 31, 20000),
                        2 ** 31 - 1 - np.arange(5000), tick * np.arange(1, 3000) - 1, tick * np.arange(1, 3000)])
    n = n[(n >= 0) & (n < 2 ** 31)].astype(object)
    assert all((x * m) >> (31 + l) == x // tick for x in n)
