"""Throughput benchmark: env steps/sec of the 2-agent MARL LOB env (MM + EXE,
2_player_fq_fqc.json), NUM_ENVS=4096 per GPU, Speed_test semantics
(gymnax_exchange/jaxen/Speed_test.py:140-224):

  master_key, *reset_keys = split(PRNGKey(0), NUM_ENVS + 1);  state0 = reset(reset_keys)
  rollout(state0, master_key, K):  per step  rng, *step_keys = split(rng, NUM_ENVS + 1)
                                             actions = per-type randint from split(step_key, n_types)
                                             env.step(step_key, state, actions, params)
  a compile run (here: W warm-up steps), then the timed run of K steps from the same
  state0 and master_key.

Before the timed run the GPU is brought to the clock it holds under sustained load (untimed,
--settle-ms, default 25 ms of back-to-back rollout steps, then state0 and master_key restored):
the chip raises its clock over the first milliseconds of load, and a 20-step timed launch
(1.3 ms) after a 5-step warm-up ran at ≈3 % lower clock than the same launch after a longer one
(profiles/r04_warmup_sensitivity.txt).  An RL training loop steps its envs back to back, so the
settled clock is the one it sees.  The JSON line reports what ran (`clock_settle`).

The K timed steps are one MARLEnv.rollout_sampled call (hftlob_env_rollout_sampled,
Speed_test's whole scan): split + sample + step fused.  By default (MARLEnv.default_slices)
that is ONE persistent k_env_rollout launch while the whole batch is resident on the GPU (the
metric: 4096 envs, 16 one-wave workgroups per CU): every env runs its K steps back to back with
its book kept in LDS, each wave's issue priority ranked by its projected finish.  Batches that
do not fit at once run as 2 contiguous env slices on their own streams, one k_env_step launch
per slice and step, so one slice's slowest envs overlap the other slice's next step (both
bit-exact with K full-batch launches, tests/test_gpu_env.py).
--mode step: Speed_test's three calls (split_keys, sample_actions, env.step) as three launches
per step.

Multi-GPU (weak scaling, one process per GPU): `--gpus N` launches N ranks itself when it is
not already running under torchrun; rank r owns envs [r*E, (r+1)*E) of ONE Speed_test rollout
over N*E envs (reset keys split(PRNGKey(0), N*E+1)[1+r*E : 1+(r+1)*E], step keys
split(master, N*E+1)[1 + r*E + e]: the reference's pmap layout, ippo_rnn_JAXMARL_pmap.py:292-332).
Day and init-state table are replicated; no collective on the data path (RCCL only for the
timing barrier and the max over ranks).  --dry-run stops before the GPU (gloo) and prints the
rank layout.  --dist-backend gloo --same-device runs the multi-rank body with every rank on
device 0 (a 1-GPU box rehearsing the N-GPU data path; --dump-state DIR writes each rank's end
state and carried key for the parity test).  Rank 0 prints ONE JSON line.
"""
import argparse
import hashlib
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "jaxmarl-hft_amd"))

NUM_ENVS = 4096
CONFIG = "2_player_fq_fqc"
PEAK_HBM_GBS = 8000.0          # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
N_CU, CLOCK_HZ = 256, 2.4e9    # MI355X CUs, max engine clock (MI355X_MICROARCH.md)
CPU_STEPS = 64                 # CPU baseline / parity: one full episode (incl. the auto-reset)
PROFILE = "r*_kernel_profile.json"  # profiles/: rocprof figures of the metric kernel (tools/profile_round.sh), newest round


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1, help="GPUs = ranks (one process per GPU)")
    ap.add_argument("--steps", type=int, default=128)
    ap.add_argument("--warmup", type=int, default=16)
    ap.add_argument("--settle-ms", type=float, default=25.0,
                    help="untimed back-to-back rollout steps (at least this much wall time) after the warm-up, "
                         "so the timed run starts at the clock the GPU holds under load; 0 = off")
    ap.add_argument("--envs", type=int, default=NUM_ENVS, help="envs per GPU")
    ap.add_argument("--n-msgs", type=int, default=400_000, help="synthetic day length (messages)")
    ap.add_argument("--mid", type=int, default=2_000_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--config", default=CONFIG, help="builtin env config (the metric: 2_player_fq_fqc)")
    ap.add_argument("--agents", default=None, help="number_of_agents_per_type override, e.g. 5,5 (Speed_test sweep)")
    ap.add_argument("--n-data-msg", type=int, default=None, help="n_data_msg_per_step override (Speed_test: 100, 1)")
    ap.add_argument("--mode", choices=("rollout", "step"), default="rollout",
                    help="rollout: one fused launch per step (key split + action sampling + step); "
                         "step: split_keys, sample_actions and env.step as three launches (SURVEY.md 8(d))")
    ap.add_argument("--slices", type=int, default=-1,
                    help="rollout mode: 0 = one persistent launch for all steps, 1..4 = env slices on streams "
                         "of their own (-1 = MARLEnv.default_slices)")
    ap.add_argument("--steps-per-call", type=int, default=0,
                    help="rollout mode: env steps per rollout_sampled call (0 = all timed steps in one call)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="CPU baseline threads (0 = the cores this process "
                                                               "may use, capped by OMP_NUM_THREADS)")
    ap.add_argument("--dry-run", action="store_true", help="rank layout only: no GPU (gloo), one JSON line")
    ap.add_argument("--dist-backend", choices=("nccl", "gloo"), default="nccl",
                    help="process group of the ranks (nccl = RCCL; gloo: the barrier / max on the CPU)")
    ap.add_argument("--same-device", action="store_true",
                    help="every rank on device 0 (with --dist-backend gloo: the N-rank body on a 1-GPU box)")
    ap.add_argument("--dump-state", default=None,
                    help="directory: each rank writes rank<r>.npz (end state, carried key) after the timed run")
    return ap.parse_args(argv)


# ------------------------------------------------------------------ launcher
def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(args) -> int:
    """`--gpus N` outside torchrun: start N rank processes (this process never touches the GPU)
    with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set, wait for all of them, and
    return the first failing exit code (the others are then terminated)."""
    n, port = args.gpus, _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    rc = 0
    while procs:
        for p in list(procs):
            code = p.poll()
            if code is None:
                continue
            procs.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in procs:
                    q.terminate()
        time.sleep(0.05)
    return rc


# ------------------------------------------------------------------ helpers
def algorithmic_bytes_per_env_step(env) -> int:
    """HBM bytes one env-step must move, from the live layout."""
    L, cfg = env.layout, env.multi_agent_config
    nO, nT, M, D = L.n_orders, L.n_trades, L.n_msgs, L.n_data_msg
    agent_words = sum(5 if k == 0 else 13 for k in L.agent_kinds)
    n_ag = len(L.agent_kinds)
    obs = sum(L.obs_dims[t] for t in L.agent_types)
    reads = 32 * D + 2 * 24 * nO + 16 + 11 * 4 + 4 * agent_words + 4 * n_ag + 8
    writes = 2 * 24 * nO + 32 * nT + 2 * 8 * M + 6 * 4 + 4 * agent_words + 4 * obs + 4 * n_ag + 4 * (1 + n_ag)
    reset = (4 * L.init_rec_words + 2 * 8 * M + 4 * (5 + agent_words + obs)) // (cfg.world_config.episode_time)
    return reads + writes + reset


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_share():
    """Host cores this process may use for the CPU baseline: its affinity set, capped by the
    cgroup CPU quota and by OMP_NUM_THREADS.  The GPU pool runs each 1-GPU job in a share of the
    host (OMP_NUM_THREADS is set to it there), while nproc / the affinity set show the whole
    machine: threads beyond the share would only time-slice.  Returns (threads, facts)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    for path, per in (("/sys/fs/cgroup/cpu.max", None), ("/sys/fs/cgroup/cpu/cpu.cfs_quota_us",
                                                        "/sys/fs/cgroup/cpu/cpu.cfs_period_us")):
        try:
            with open(path) as f:
                q = f.read().split()
            if per is None:
                if q and q[0] != "max":
                    quota = int(q[0]) / int(q[1])
            else:
                with open(per) as f:
                    p = int(f.read().split()[0])
                if int(q[0]) > 0:
                    quota = int(q[0]) / p
            break
        except (OSError, ValueError, IndexError):
            continue
    omp = os.environ.get("OMP_NUM_THREADS")
    thr = aff
    if quota:
        thr = min(thr, max(1, int(quota)))
    if omp and omp.isdigit() and int(omp) > 0:
        thr = min(thr, int(omp))
    return thr, {"affinity_cores": aff, "cgroup_quota_cores": quota, "omp_num_threads": omp}


def _profile(pattern):
    """The newest round's profile summary (profiles/rNN_kernel_profile.json), with its file name."""
    import glob
    found = sorted(glob.glob(os.path.join(ROOT, "profiles", pattern)))
    if not found:
        return None
    with open(found[-1]) as f:
        return dict(json.load(f), file=os.path.join("profiles", os.path.basename(found[-1])))


def timed_window(K: int, max_steps: int, ctr0: int = 0) -> str:
    """Which steps of each env's episode the K timed steps cover: Speed_test's timed rollout starts
    from the reset state (step counter 0), and an env's episode ends on the step whose counter
    satisfies max_steps - step - 1 <= 1 (marl_env.py:711-718 _episode_done_time, then the auto-reset :787-803)."""
    ends, ctr = [], ctr0
    for t in range(K):
        if max_steps - ctr - 1 <= 1:
            ends.append(t)
            ctr = 0
        else:
            ctr += 1
    what = (f"{len(ends)} episode end(s) with auto-reset, at timed step(s) {ends}" if ends
            else "no episode end (the auto-reset and the episode-end trades are outside the window)")
    return f"timed steps 0-{K - 1} from the reset state (step counter {ctr0}), {max_steps}-step episodes: {what}"


def compare_states(env, cpu, gpu) -> str:
    """Integer words of the record bit-exact, float words within 1e-5."""
    import numpy as np
    L = env.layout
    fw = [L.off_world + 3, L.off_world + 4]
    for k, off in zip(L.agent_kinds, L.agent_offsets):
        fw += [off + 3, off + 4] if k == 0 else [off + j for j in (0, 4, 5, 6, 7, 8, 9, 10, 11, 12)]
    mask = np.ones(cpu.shape[1], bool)
    mask[fw] = False
    bad = int(((cpu != gpu) & mask[None, :]).sum())
    if bad:
        raise AssertionError(f"cpu_baseline parity: {bad} integer state words differ between the CPU oracle and "
                             "the GPU rollout")
    if not np.allclose(cpu[:, fw].view(np.float32), gpu[:, fw].view(np.float32), rtol=1e-5, atol=1e-5,
                       equal_nan=True):
        raise AssertionError("cpu_baseline parity: float state words differ beyond 1e-5")
    return (f"end state of the {cpu.shape[0]}-env x {CPU_STEPS}-step rollout == the GPU's: "
            f"{int(mask.sum())} int words/env bit-exact, {len(fw)} float words/env within 1e-5")


def cpu_baseline(env, day, state0, master0, n_threads):
    """The plain-C restatement (oracle/oracle.c, test infrastructure) built -O3 -march=native on
    this host, its Speed_test rollout loop in C, timed on this host's cores: the metric workload
    (4096 envs x one 64-step episode) on n_threads cores and on 1 core.  Returns the line's
    object and the end state (for the parity check against the GPU)."""
    import numpy as np
    sys.path.insert(0, ROOT)
    from oracle import pyoracle as O
    model = _cpu_model()
    tag = hashlib.sha1((model + open(os.path.join(ROOT, "oracle", "oracle.c")).read()).encode()).hexdigest()[:12]
    L = O.native_lib(f"/tmp/hftlob_oracle_native_{tag}.so")
    c, msgs, init = env.cfg_c, day.msgs, env._init_states.cpu().numpy()
    st0 = state0.cpu().numpy()
    m0 = master0.cpu().numpy().view(np.uint32)
    E = st0.shape[0]
    thr = L.oracle_set_threads(n_threads)
    t0 = time.perf_counter()
    st, _ = O.rollout_sampled(c, m0, msgs, init, st0, CPU_STEPS, L=L)
    v = E * CPU_STEPS / (time.perf_counter() - t0)
    L.oracle_set_threads(1)
    t0 = time.perf_counter()
    st1, _ = O.rollout_sampled(c, m0, msgs, init, st0, CPU_STEPS, L=L)
    v1 = E * CPU_STEPS / (time.perf_counter() - t0)
    _, facts = cpu_share()
    aff = facts["affinity_cores"]
    v_aff = None
    if aff > thr:  # every core the affinity set shows (beyond the job's quota the threads time-slice)
        L.oracle_set_threads(aff)
        t0 = time.perf_counter()
        st_aff, _ = O.rollout_sampled(c, m0, msgs, init, st0, CPU_STEPS, L=L)
        v_aff = E * CPU_STEPS / (time.perf_counter() - t0)
        if not (st_aff == st).all():
            raise AssertionError("cpu_baseline: the all-affinity-cores and quota-thread CPU rollouts differ")
    L.oracle_set_threads(thr)
    if not (st1 == st).all():
        raise AssertionError("cpu_baseline: 1-thread and multi-thread CPU rollouts differ")
    eff = v / (thr * v1) if thr and v1 else None
    return {"value": round(v, 1), "unit": "env steps/s", "cores": thr, "kind": "port",
            "sample": (f"{E} envs x {CPU_STEPS} steps (one episode incl. auto-reset) of the metric config/day/seeds, "
                       "Speed_test rollout loop in C (oracle/oracle.c oracle_rollout_sampled), "
                       f"gcc -O3 -march=native, OpenMP {thr} threads"),
            "single_core_value": round(v1, 1), "single_core_sample": f"the same {E} x {CPU_STEPS} workload, 1 thread",
            "thread_scaling_efficiency": round(eff, 3) if eff else None,
            "all_affinity_cores_value": round(v_aff, 1) if v_aff else None,
            "all_affinity_cores_sample": (f"the same {E} x {CPU_STEPS} workload on {aff} OpenMP threads (every core "
                                          "of the affinity set; the job's cgroup quota caps the CPU time)")
            if v_aff else None,
            "cores_rule": ("threads = this job's host CPU share: the affinity set capped by the cgroup quota and "
                           "OMP_NUM_THREADS (bench.py cpu_share)"),
            "cpu_model": model, "nproc": os.cpu_count(), **facts}, st


# ------------------------------------------------------------------ rank body
def dry_run(args):
    """Rank layout without the GPU: gloo process group, each rank's env block and key rows."""
    from hftlob import dist as D
    R = D.init_from_env("gloo")
    E = args.envs
    a, b = D.env_slice(R.rank, E)
    mine = {"rank": R.rank, "envs": [a, b], "reset_key_rows": [1 + a, 1 + b], "key_e0": a, "key_n": R.world * E}
    gathered = [mine]
    if R.dist is not None:
        gathered = [None] * R.world
        R.dist.all_gather_object(gathered, mine)
    if R.rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": R.world, "num_envs_per_gpu": E,
                          "num_envs_total": R.world * E, "ranks": sorted(gathered, key=lambda g: g["rank"])}))
    D.finalize(R)


def main(argv=None):
    args = parse_args(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch(args)
    if args.dry_run:
        return dry_run(args)
    import numpy as np
    import torch
    from hftlob import dist as D
    if args.same_device and args.dist_backend != "gloo":
        raise SystemExit("bench: --same-device needs --dist-backend gloo (RCCL takes one GPU per rank)")
    R = D.init_from_env(args.dist_backend)
    world, rank, local = R.world, R.rank, (0 if args.same_device else R.local)
    if world != args.gpus:
        print(f"bench: WORLD_SIZE={world} overrides --gpus {args.gpus}", file=sys.stderr)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    red_dev = dev if args.dist_backend == "nccl" else None  # where max_over_ranks reduces

    import dataclasses
    from hftlob.config_io import builtin_config
    from hftlob.data.synthetic import LobsterDay, generate_day
    from hftlob.env import MARLEnv, split_keys

    cfg = builtin_config(args.config)
    if args.agents:
        cfg = dataclasses.replace(cfg, number_of_agents_per_type=[int(x) for x in args.agents.split(",")])
    if args.n_data_msg:
        cfg = dataclasses.replace(cfg, world_config=dataclasses.replace(cfg.world_config,
                                                                        n_data_msg_per_step=args.n_data_msg))
    w = cfg.world_config
    snap = w.n_data_msg_per_step * w.start_resolution
    cache = f"/tmp/hftlob_day_{args.n_msgs}_{args.mid}_{snap}.npz"
    if local == 0 and not os.path.exists(cache):
        d = generate_day(n_msgs=args.n_msgs, mid=args.mid, snap_every=snap)
        np.savez(cache + f".{os.getpid()}.npz", msgs=d.msgs, books=d.books, snap_idx=d.snap_idx, tick=d.tick_size)
        os.replace(cache + f".{os.getpid()}.npz", cache)
    D.barrier(R)
    z = np.load(cache)
    day = LobsterDay(msgs=z["msgs"], books=z["books"], snap_idx=z["snap_idx"], tick_size=int(z["tick"]))

    E = args.envs
    env = MARLEnv(None, cfg, data=day, device=dev, return_info=False, persistent_outputs=True)
    params = env.default_params
    # Speed_test: master_key, *reset_keys = split(PRNGKey(0), NUM_ENVS + 1), NUM_ENVS = world * E
    all_keys = split_keys(torch.zeros((1, 2), dtype=torch.int32, device=dev), world * E + 1)[0]
    master0 = all_keys[0].clone()
    _, state = env.reset(D.rank_keys(all_keys, rank, E).contiguous(), params)
    state0 = state.buf.clone()
    max_steps = int(state.world_state.max_steps_in_episode[0].item())
    ctr0 = int(state.world_state.step_counter[0].item())
    key_e0, key_n = rank * E, world * E
    if args.slices < 0:
        args.slices = env.default_slices(E)
    if args.mode == "rollout":
        env.prepare_rollout(args.slices)
    T = (args.steps_per_call if args.steps_per_call > 0 else max(args.steps, 1)) if args.mode == "rollout" else 1
    kbuf = [master0.clone(), torch.empty(2, dtype=torch.int32, device=dev)]
    nstep = [0]

    def run(n_steps):  # n_steps env steps continuing the rollout from (state, kbuf)
        while n_steps > 0:
            n, k = min(T, n_steps), nstep[0]
            if args.mode == "rollout":
                env.rollout_sampled(kbuf[k % 2], kbuf[(k + 1) % 2], state, params, n, n_slices=args.slices,
                                    key_e0=key_e0, key_n=key_n)
            else:  # Speed_test's three calls, each its own launch: split, Discrete.sample, env.step
                ks = split_keys(kbuf[k % 2].reshape(1, 2), key_n + 1)[0]
                kbuf[(k + 1) % 2].copy_(ks[0])
                sk = ks[1 + key_e0:1 + key_e0 + E].contiguous()
                env.step(sk, state, env.sample_actions(sk), params)
            nstep[0] = k + 1
            n_steps -= n

    def restart():  # rollout(state0, master_key): back to the reset state and the master key
        state.buf.copy_(state0)
        kbuf[0].copy_(master0)
        nstep[0] = 0

    stream = torch.cuda.current_stream(dev)

    def timed():  # the K timed steps from (state0, master0): barrier + sync on both sides, max over ranks
        restart()
        torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        D.barrier(R)
        torch.cuda.synchronize()
        D.barrier(R)
        t0 = time.perf_counter()
        ev0.record(stream)                    # on the launch stream (slice 0 runs on it; the others join it)
        run(args.steps)
        ev1.record(stream)
        torch.cuda.synchronize()
        D.barrier(R)
        el = time.perf_counter() - t0
        return D.max_over_ranks(R, el, device=red_dev), ev0.elapsed_time(ev1) / args.steps

    run(args.warmup)                          # Speed_test's compile run
    # the same K steps timed right after the warm-up, as Speed_test times them (reported beside
    # `value` as `unsettled`: the GPU has not reached its loaded clock yet)
    uns_elapsed, uns_kern_ms = timed() if args.settle_ms > 0 else (None, None)
    # clock settle (untimed): calls of the timed run's length (T steps, so every launch a profiler
    # sees is the timed shape) until --settle-ms of wall time has passed, then back to state0 /
    # master_key; the timed run below is unchanged by it (same state, same K steps)
    torch.cuda.synchronize()
    settle_steps, ts0 = 0, time.perf_counter()
    while args.settle_ms > 0 and (time.perf_counter() - ts0) * 1e3 < args.settle_ms and settle_steps < 16384:
        run(T)
        settle_steps += T
        torch.cuda.synchronize()
    settle_ms = (time.perf_counter() - ts0) * 1e3
    elapsed, kern_ms = timed()                # kern_ms: HIP-event time of the timed region per batched step
    if args.dump_state:  # this rank's end state and carried key (tests/test_gpu_bench_ranks.py)
        os.makedirs(args.dump_state, exist_ok=True)
        np.savez(os.path.join(args.dump_state, f"rank{rank}.npz"), state=state.buf.cpu().numpy(),
                 key=kbuf[nstep[0] % 2].cpu().numpy(), key_e0=key_e0, key_n=key_n, steps=args.steps)

    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        thr = args.cpu_threads or cpu_share()[0]
        cpu, cpu_state = cpu_baseline(env, day, state0, master0, thr)
        restart()                             # the same rollout on the GPU, for the parity check
        run(CPU_STEPS)
        torch.cuda.synchronize()
        cpu["parity"] = compare_states(env, cpu_state, state.buf.cpu().numpy())
    if rank != 0:
        D.finalize(R)
        return 0
    value = world * E * args.steps / elapsed
    per_env = algorithmic_bytes_per_env_step(env)
    achieved = per_env * E / (kern_ms * 1e-3) / 1e9
    metric_cfg = args.config == CONFIG and not args.agents and not args.n_data_msg
    prof = _profile(PROFILE) if metric_cfg and args.mode == "rollout" else None
    if prof and prof.get("slices", 2) != args.slices:  # measured on another launch shape
        prof = None
    kernel = "k_env_rollout" if args.mode == "rollout" and args.slices == 0 else "k_env_step"
    # the profile's figures for this run's launch length (HBM bytes per env-step depend on it: the
    # persistent launch loads the books once per launch); the nearest measured length otherwise
    traffic, t_spl, rp = None, None, None
    if prof:
        by = prof.get("hbm_bytes_per_env_step_by_launch_steps") or (
            {str(prof.get("traffic_steps_per_launch", prof.get("steps_per_launch", 1))): prof["hbm_bytes_per_env_step"]}
            if prof.get("hbm_bytes_per_env_step") else {})
        if by:
            t_spl = min(by, key=lambda k: abs(int(k) - T))
            traffic = round(by[t_spl] * E)
            t_spl = int(t_spl)
        rp = {k: prof[k] for k in ("kernel_avg_us", "launches", "steps_per_launch", "kernel_us_per_step",
                                   "envs_per_launch", "launches_in_flight", "source") if k in prof}
        r20 = prof.get("rocprof_20_step_launch")
        if r20 and abs(T - 20) < abs(T - rp.get("steps_per_launch", T)):
            rp = dict(rp, **r20)
    # "hbm" is the normative roofline: the reference's per-step state I/O priced at
    # the HBM peak.  The kernel does not run against it (limiter: issue and dependent latency)
    roofline = {"bound": "hbm", "bound_kind": "normative: algorithmic bytes at HBM peak, not the limiter",
                "achieved": round(achieved, 2), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": round(achieved / PEAK_HBM_GBS, 5), "traffic": traffic,
                "kernel": kernel, "kernel_ms": round(kern_ms, 5), "bytes_per_env_step": per_env,
                "units_per_launch": E,
                "launches_per_step": (args.slices or round(1 / T, 6)) if args.mode == "rollout" else 3,
                "limiter": ("issue / dependent latency, not HBM: the counted traffic is far below the algorithmic "
                            "bytes (the books stay in LDS) and below the peak (counted_traffic_frac); see "
                            "issue_roofline and DESIGN.md section 4")}
    if traffic is not None:
        roofline["traffic_steps_per_launch"] = t_spl
        roofline["traffic_source"] = {"file": prof.get("file"), "run": prof.get("source"),
                                      "commit": prof.get("commit")}
        if t_spl == T:  # the counted HBM bytes of a launch of this run's length / this run's time per step
            roofline["counted_traffic_frac"] = round(traffic / (kern_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 5)
    issue = None
    if prof:
        roofline["rocprof"] = rp
        if prof.get("salu_per_env_step"):
            # the CU's one scalar ALU, shared by its waves, is the scarcest pipe;
            # SALU per env-step from the SQ pass over the launch length nearest this run's
            sby = prof.get("salu_per_env_step_by_launch_steps") or {
                str(prof.get("traffic_steps_per_launch", prof.get("steps_per_launch", T))): prof["salu_per_env_step"]}
            s_spl = min(sby, key=lambda k: abs(int(k) - T))
            prof = dict(prof, salu_per_env_step=sby[s_spl], traffic_steps_per_launch=int(s_spl))
            a = prof["salu_per_env_step"] * world * E * args.steps / elapsed / N_CU / world
            issue = {"bound": "salu_issue", "achieved": round(a / 1e9, 4), "peak": CLOCK_HZ / 1e9,
                     "unit": "G SALU instr/s per CU", "frac": round(a / CLOCK_HZ, 4),
                     "salu_per_env_step": prof["salu_per_env_step"], "source": prof.get("source"),
                     "salu_steps_per_launch": prof.get("traffic_steps_per_launch", prof.get("steps_per_launch"))}
    workload = (f"{CONFIG}.json MM fixed_quants + EXE fixed_quants_complex, {env.num_msgs_per_step} msgs/step, "
                "Speed_test semantics (auto-reset on)" if metric_cfg else
                f"{args.config if args.config == 'default' else args.config + '.json'} "
                f"agents {list(cfg.number_of_agents_per_type)}, {env.num_msgs_per_step} msgs/step, "
                "Speed_test semantics (auto-reset on)")
    line = {
        "metric": "env steps/sec (whole node), 2-agent MARL, 10-level LOB, NUM_ENVS=4096",
        "value": round(value, 1),
        "unit": "env steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        # untimed steps the GPU ran before the timed K: the W warm-up, the unsettled timing run and the settle
        "warmup_effective": args.warmup + (args.steps if uns_elapsed is not None else 0) + settle_steps,
        "clock_settle": {"steps": settle_steps, "ms": round(settle_ms, 1), "untimed": True,
                         "then": "state0 and master_key restored; the timed run starts from them"},
        "unsettled": ({"value": round(world * E * args.steps / uns_elapsed, 1),
                       "ms_per_step": round(uns_elapsed / args.steps * 1e3, 4),
                       "kernel_ms": round(uns_kern_ms, 5),
                       "what": (f"the same {args.steps} steps from state0 timed right after the {args.warmup} "
                                "warm-up steps, before the clock settle (Speed_test's order; --settle-ms 0 "
                                "makes this the value)")} if uns_elapsed is not None else None),
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": f"synthetic LOBSTER day ({args.n_msgs} msgs, PCG64 seed 20260403, mid {args.mid})",
        "config": {"workload": workload, "num_envs_per_gpu": E, "num_envs_total": world * E,
                   "parallelism": f"dp{world} (env shards of one {world * E}-env Speed_test rollout)",
                   "launch": ((f"one persistent k_env_rollout launch of {T} steps per rollout_sampled call "
                               "(every env's steps back to back, its book kept in LDS)" if args.slices == 0 else
                               f"{args.slices} env slices on their own streams, {T} steps per rollout_sampled call")
                              if args.mode == "rollout" else "split_keys + sample_actions + env.step per step"),
                   "mode": args.mode, "seeds": "Speed_test: split(PRNGKey(0), NUM_ENVS + 1)",
                   "timed_window": timed_window(args.steps, max_steps, ctr0)},
        "roofline": roofline,
        "issue_roofline": issue,
        "cpu_baseline": cpu,
    }
    print(json.dumps(line))
    D.finalize(R)
    return 0


if __name__ == "__main__":
    sys.exit(main())
