"""Run lengths of the metric workload's message classes, from the CPU oracle built with
-DORACLE_STATS (its per-message class trace): how many consecutive processed messages could be
handled as one lane-parallel batch.  Usage: python tools/msg_runs.py [n_envs] [n_steps]"""
import ctypes as C
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "jaxmarl-hft_amd")]
import numpy as np  # noqa: E402

CLS = ["doNothing", "add behind/at best", "add improving best", "crossing add", "add into full side",
       "cancel qty 0", "cancel by id", "cancel by init id", "cancel no row, last empty", "cancel no row, last used",
       "no row, last empty, init row < qty"]


def main():
    E = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    lib = "/tmp/liboracle_trace.so"
    subprocess.run(["gcc", "-O2", "-DORACLE_STATS", "-ffp-contract=off", "-shared", "-fPIC", "-o", lib,
                    os.path.join(ROOT, "oracle", "oracle.c"), "-lm"], check=True)
    from oracle import pyoracle as O
    from hftlob.config_io import builtin_config
    from hftlob.data.synthetic import generate_day
    from hftlob.data.windows import make_windows
    from hftlob.layout import pack_env_cfg
    L = O._bind(C.CDLL(lib))
    L.oracle_set_threads(1)
    cfg = builtin_config("2_player_fq_fqc")
    w = cfg.world_config
    day = generate_day(n_msgs=400_000, mid=2_000_000, snap_every=w.n_data_msg_per_step * w.start_resolution)
    win = make_windows(day, w)
    c, lay = pack_env_cfg(cfg, len(win.starts), day.msgs.shape[0], True)
    init = O.init_states(c.lob, win, day.msgs, w, lay.init_rec_words)
    keys = O.split_keys(np.zeros((1, 2), np.uint32), E + 1)[0]
    st, _ = O.env_reset(c, keys[1:], init)
    C.c_longlong.in_dll(L, "oracle_trace_n").value = 0
    O.rollout_sampled(c, keys[0], day.msgs, init, st, T, L=L)
    n = C.c_longlong.in_dll(L, "oracle_trace_n").value
    tr = np.ctypeslib.as_array((C.c_byte * n).in_dll(L, "oracle_trace")).astype(np.int64)
    M = lay.n_msgs
    print(f"{E} envs x {T} steps x {M} msgs: {n} messages (expected {E * T * M})")
    for k, name in enumerate(CLS):
        print(f"  {k} {name:28s} {np.mean(tr == k) * 100:6.2f} %")
    seq = tr.reshape(-1, M)  # per env-step (the oracle runs env by env, step by step)
    runs = []
    for row in seq:
        live = row[~np.isin(row, (0, 5, 8, 10))]   # the kernel skips these (10: only with an exact init test)
        r = 0
        for v in live:
            if v == 1:
                r += 1
            else:
                if r:
                    runs.append(r)
                r = 0
        if r:
            runs.append(r)
    runs = np.array(runs)
    live_n = np.sum(~np.isin(tr, (0, 5, 8, 10)))
    st = tr.reshape(-1, M)
    T_ = st.shape[0] // E
    by_step = np.array([np.mean(st.reshape(E, T_, M)[:, t] == 10) for t in range(T_)]) * M
    print("class-10 messages per env-step by episode step:", np.round(by_step[:20], 2).tolist())
    print(f"processed messages per step: {live_n / len(seq):.1f}; simple adds per step {np.sum(tr == 1) / len(seq):.1f}")
    print(f"runs of simple adds: {len(runs) / len(seq):.1f} per step, mean length {runs.mean():.2f}; "
          f"length histogram {np.bincount(runs)[1:12].tolist()}")


if __name__ == "__main__":
    main()
