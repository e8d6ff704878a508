"""Message mix of the metric workload, from the CPU oracle built with -DORACLE_STATS:
which handler each message takes and what happens in it (guides the kernel's fast paths).
Usage: python tools/msg_mix.py [n_envs] [n_steps]"""
import ctypes as C
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "jaxmarl-hft_amd")]
import numpy as np  # noqa: E402

NAMES = {0: "ask_lim", 1: "bid_lim", 2: "cancel ask", 3: "cancel bid", 4: "noop", 5: "type 4 (exec)",
         6: "lim with qty <= 0", 7: "lim that crosses (>= 1 match)", 10: "cancels", 11: "cancel qty 0",
         12: "cancel found by oid", 13: "cancel removes the row", 14: "cancel at the best price",
         15: "best ask price changed", 16: "best bid price changed", 17: "best ask (p,q) changed",
         18: "best bid (p,q) changed", 20: "match trips", 21: "cancel found by the init-id fallback",
         22: "cancel of no row (wraps to the last slot)", 23: "... and the last slot is empty",
         24: "match trips that empty the top order",
         25: "limit order into a full side (check_book_fill eviction)"}


def main():
    E = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    lib = "/tmp/liboracle_stats.so"
    subprocess.run(["gcc", "-O2", "-DORACLE_STATS", "-ffp-contract=off", "-shared", "-fPIC", "-o", lib,
                    os.path.join(ROOT, "oracle", "oracle.c"), "-lm"], check=True)
    from oracle import pyoracle as O
    from hftlob.config_io import builtin_config
    from hftlob.data.synthetic import generate_day
    from hftlob.data.windows import make_windows
    from hftlob.layout import pack_env_cfg
    L = O._bind(C.CDLL(lib))
    cfg = builtin_config("2_player_fq_fqc")
    w = cfg.world_config
    day = generate_day(n_msgs=100_000, snap_every=w.n_data_msg_per_step * w.start_resolution)
    win = make_windows(day, w)
    c, lay = pack_env_cfg(cfg, len(win.starts), day.msgs.shape[0], True)
    init = O.init_states(c.lob, win, day.msgs, w, lay.init_rec_words)
    keys = O.split_keys(np.zeros((1, 2), np.uint32), E + 1)[0]
    st, _ = O.env_reset(c, keys[1:], init)
    stats = (C.c_longlong * 32).in_dll(L, "oracle_stats")
    for i in range(32):
        stats[i] = 0
    O.rollout_sampled(c, keys[0], day.msgs, init, st, T, L=L)
    n = E * T * lay.n_msgs
    print(f"{E} envs x {T} steps x {lay.n_msgs} msgs = {n} messages")
    for i, name in NAMES.items():
        print(f"  {name:32s} {stats[i]:10d}  {stats[i] / n * 100:6.2f} % of messages")


if __name__ == "__main__":
    main()
