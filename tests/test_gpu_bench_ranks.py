"""bench.py's multi-rank body on ONE GPU: `--gpus 2 --dist-backend gloo --same-device` starts two
rank processes (the launcher of the N-GPU bench) that both run on device 0, with the gloo group
for the timing barrier and the max over ranks.  Rank r steps envs [r*E, (r+1)*E) of one
Speed_test rollout over 2E envs (reset keys split(PRNGKey(0), 2E + 1)[1 + r*E:], step keys
split(master, 2E + 1)[1 + r*E + e]: key_e0 = r*E, key_n = 2E; ippo_rnn_JAXMARL_pmap.py:292-332).
Each rank's end state and carried key must equal the CPU oracle's rollout of its block: the
N-GPU data path (C4/C5) exercised on hardware before an 8-GPU node runs it."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from hftlob.config_io import builtin_config
from hftlob.data.synthetic import generate_day
from hftlob.data.windows import make_windows
from hftlob.layout import pack_env_cfg
from oracle import pyoracle as O
from test_gpu_env import _float_words

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("slices", [0, 2])
def test_bench_two_ranks_same_device(slices, tmp_path):
    E, T, N_MSGS = 256, 66, 30_000
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--envs", str(E), "--steps", str(T),
           "--warmup", "2", "--n-msgs", str(N_MSGS), "--no-cpu-baseline", "--dist-backend", "gloo",
           "--same-device", "--slices", str(slices), "--dump-state", str(tmp_path)]
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["config"]["num_envs_total"] == 2 * E and line["steps"] == T
    assert line["value"] > 0

    cfg = builtin_config("2_player_fq_fqc")
    w = cfg.world_config
    day = generate_day(n_msgs=N_MSGS, mid=2_000_000, snap_every=w.n_data_msg_per_step * w.start_resolution)
    win = make_windows(day, w)
    c, L = pack_env_cfg(cfg, len(win.starts), day.msgs.shape[0], True)
    init = O.init_states(c.lob, win, day.msgs, w, L.init_rec_words)
    keys = O.split_keys(np.zeros((1, 2), np.uint32), 2 * E + 1)[0]
    fw = _float_words(type("E", (), {"layout": L})())
    mask = np.ones(L.rec_words, bool)
    mask[fw] = False
    for rank in range(2):
        got = np.load(tmp_path / f"rank{rank}.npz")
        assert int(got["key_e0"]) == rank * E and int(got["key_n"]) == 2 * E
        st0, _ = O.env_reset(c, keys[1 + rank * E:1 + (rank + 1) * E], init)
        o_end, o_key = O.rollout_sampled(c, keys[0], day.msgs, init, st0, T, key_e0=rank * E, key_n=2 * E)
        g = got["state"]
        bad = np.argwhere((o_end != g) & mask[None, :])
        assert bad.size == 0, f"rank {rank}: int words differ at {bad[:5].tolist()}"
        assert np.allclose(o_end[:, fw].view(np.float32), g[:, fw].view(np.float32), rtol=1e-5, atol=1e-5)
        assert (got["key"].view(np.uint32) == o_key).all(), f"rank {rank}: carried key"
