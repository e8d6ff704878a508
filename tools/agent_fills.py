"""How often each agent of the metric config has a fill in a step, and how many trades a step
logs (guides the rewards' no-fill path and the trade view's register sets): the C oracle's
debug trades over 128 envs x 40 Speed_test steps.  Usage: python tools/agent_fills.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "jaxmarl-hft_amd")]
import numpy as np  # noqa: E402
from oracle import pyoracle as O  # noqa: E402
from hftlob.config_io import builtin_config  # noqa: E402
from hftlob.data.synthetic import generate_day  # noqa: E402
from hftlob.data.windows import make_windows  # noqa: E402
from hftlob.layout import pack_env_cfg, trader_ids  # noqa: E402

cfg = builtin_config("2_player_fq_fqc")
w = cfg.world_config
day = generate_day(n_msgs=400_000, mid=2_000_000, snap_every=w.n_data_msg_per_step * w.start_resolution)
win = make_windows(day, w)
c, lay = pack_env_cfg(cfg, len(win.starts), day.msgs.shape[0], True)
init = O.init_states(c.lob, win, day.msgs, w, lay.init_rec_words)
E, T = 128, 40
keys = O.split_keys(np.zeros((1, 2), np.uint32), E + 1)[0]
st, _ = O.env_reset(c, keys[1:], init)
tids = [t for ids in trader_ids(cfg) for t in ids]
m = keys[0]
hits, ntr = np.zeros(len(tids)), []
for k in range(T):
    ks = O.split_keys(m[None], E + 1)[0]
    m, sk = ks[0], ks[1:]
    res = O.env_step(c, sk, O.sample_actions(c, sk), day.msgs, init, st, debug=True)
    st, dbg = res[0], res[-1]
    tr = dbg[:, 40:].reshape(E, -1, 8)
    valid = tr[:, :, 0] >= 0
    ntr.append(valid.sum(1))
    for a, t in enumerate(tids):
        hits[a] += (valid & ((tr[:, :, 6] == t) | (tr[:, :, 7] == t))).any(1).sum()
ntr = np.concatenate(ntr)
print(f"trader ids {tids}: share of env-steps with a fill {np.round(hits / (E * T), 4).tolist()}")
print(f"trades per step: mean {ntr.mean():.1f}, max {ntr.max()}, share above 63: {(ntr > 63).mean():.4f}")
