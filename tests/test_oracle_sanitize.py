"""The CPU oracle under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md section 5:
sanitizers on the CPU restatement), and its C rollout loop (bench.py's CPU baseline and the
metric-shape parity tests) against per-step calls.

oracle/sanitize_main.c drives reset, one env step with info, a rollout across an auto-reset and
the engine operator on real packed configs; any out-of-bounds access, overflow of the fixed-size
stack buffers or undefined behaviour aborts it (-fno-sanitize-recover=all).  Its outputs must
equal the -O2 oracle's bit for bit."""
import os
import subprocess

import numpy as np
import pytest

from hftlob.config_io import builtin_config
from hftlob.data.synthetic import generate_day
from hftlob.data.windows import make_windows
from hftlob.layout import pack_env_cfg
from oracle import pyoracle as O
from test_gpu_env import variant

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(ROOT, "oracle", "_build", "oracle_san")


def _setup(cfg, n_msgs=20_000, seed=12):
    w = cfg.world_config
    day = generate_day(n_msgs=n_msgs, seed=seed, snap_every=w.n_data_msg_per_step * w.start_resolution)
    win = make_windows(day, w)
    c, L = pack_env_cfg(cfg, len(win.starts), day.msgs.shape[0], True)
    init = O.init_states(c.lob, win, day.msgs, w, L.init_rec_words)
    return c, L, day, init


@pytest.fixture(scope="module")
def san_exe():
    r = subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "-s", "san"], capture_output=True, text=True)
    if r.returncode != 0:
        pytest.skip(f"sanitizer build unavailable: {r.stderr[-400:]}")
    return SAN


@pytest.mark.parametrize("name,agents,changes", [("2_player_fq_fqc", None, None),
                                                 ("3_player_fq_fqc_dir", [2, 2, 3], None),
                                                 ("mm_debug_fixed_quant", None, None),
                                                 ("2_player_fq_fqc", [3, 2],
                                                  dict(action_space="fixed_prices", n_actions=4, fixed_quant_value=7))])
def test_oracle_under_asan_ubsan(san_exe, tmp_path, name, agents, changes):
    import dataclasses
    cfg = builtin_config(name)
    if changes:
        cfg = variant(cfg, "Execution", **changes)
    if agents:
        cfg = dataclasses.replace(cfg, number_of_agents_per_type=agents)
    c, L, day, init = _setup(cfg)
    E, T, BE = 12, 66, 6
    keys = np.arange(2 * E, dtype=np.uint32).reshape(E, 2) * 7 + 3
    master = np.array([5, 9], np.uint32)
    rng = np.random.default_rng(3)
    book = day.msgs[rng.integers(0, day.msgs.shape[0] - 200, BE)[:, None] + np.arange(150)[None, :]].astype(np.int32)
    d = tmp_path
    (d / "cfg.bin").write_bytes(bytes(c))
    day.msgs.astype(np.int32).tofile(d / "msgs.bin")
    np.ascontiguousarray(init, np.int32).tofile(d / "init.bin")
    keys.tofile(d / "keys.bin")
    book.tofile(d / "book.bin")
    (d / "params.txt").write_text(f"{E} {T} {master[0]} {master[1]} {BE} {book.shape[1]}\n")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([san_exe, str(d)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    # same results as the -O2 checker
    st, _ = O.env_reset(c, keys, init)
    acts = O.sample_actions(c, keys)
    st, _, _, _, _, info = O.env_step(c, keys, acts, day.msgs, init, st)
    st, _ = O.rollout_sampled(c, master, day.msgs, init, st, T)
    assert (np.fromfile(d / "state.bin", np.int32).reshape(st.shape) == st).all()
    assert (np.fromfile(d / "info.bin", np.int32).reshape(info.shape) == info).all()
    nO, nT = c.lob.n_orders, c.lob.n_trades
    a0 = np.full((BE, nO, 6), -1, np.int32)
    t0 = np.full((BE, nT, 8), -1, np.int32)
    a, b, t, ba, bb = O.book_process(c.lob, book, a0, a0, t0)
    got = np.fromfile(d / "book_out.bin", np.int32)
    want = np.concatenate([a.ravel(), b.ravel(), t.ravel(), ba.ravel(), bb.ravel()])
    assert (got == want).all()


def test_c_rollout_equals_per_step_calls():
    """oracle_rollout_sampled (the C loop) == split + Discrete.sample + env_step per step, and a
    rank's shard (key_e0, key_n) == its rows of the whole-batch rollout."""
    cfg = builtin_config("2_player_fq_fqc")
    c, L, day, init = _setup(cfg)
    E, T = 10, 67
    keys = O.split_keys(np.array([[0, 0]], np.uint32), E + 1)[0]
    master0, st0 = keys[0], O.env_reset(c, keys[1:], init)[0]
    st, master = st0.copy(), master0.copy()
    for _ in range(T):
        ks = O.split_keys(master[None], E + 1)[0]
        master, sk = ks[0].copy(), ks[1:].copy()
        st = O.env_step(c, sk, O.sample_actions(c, sk), day.msgs, init, st, with_info=False)[0]
    got, m = O.rollout_sampled(c, master0, day.msgs, init, st0, T)
    assert (got == st).all() and (m == master).all()
    half, m2 = O.rollout_sampled(c, master0, day.msgs, init, st0[4:], T, key_e0=4, key_n=E)
    assert (half == st[4:]).all() and (m2 == master).all()
