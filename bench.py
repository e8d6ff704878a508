"""Throughput benchmark: env steps/sec of the 2-agent MARL LOB env (MM + EXE,
2_player_fq_fqc.json), NUM_ENVS=4096 per GPU, Speed_test semantics
(gymnax_exchange/jaxen/Speed_test.py:140-224):

  per step:  rng, *step_keys = split(rng, NUM_ENVS + 1)
             actions = per-type randint from split(step_key, n_types)
             env.step(step_key, state, actions, params)
  all three in ONE HIP launch (MARLEnv.step_sampled -> hftlob_env_step_sampled);
  the unfused three-launch form is checked bit-exact against it in
  tests/test_gpu_env.py.

Launches (default): the K timed steps are one MARLEnv.rollout_sampled call
(hftlob_env_rollout_sampled, Speed_test's whole scan): the 4096 envs run as 2
contiguous slices, each stepped by its own k_env_step launches on its own
stream, so one slice's slowest envs overlap the other slice's next step
instead of idling CUs at every step boundary (bit-exact with K full-batch
launches, tests/test_gpu_env.py).  --slices 0: one full-batch
hftlob_env_step_sampled launch per step (--graph-steps G > 0 replays a
captured HIP graph of G such launches).  roofline.kernel_ms is the HIP-event
time of the timed region on the caller's stream / K.

Weak scaling: every rank (one process per GPU) steps its own 4096 envs on a
replicated synthetic LOBSTER day; no collective on the data path (only the
timing barrier / max-over-ranks).  Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "jaxmarl-hft_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

NUM_ENVS = 4096
CONFIG = "2_player_fq_fqc"
PEAK_HBM_GBS = 8000.0          # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


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


def cpu_baseline(env, day, n_envs, n_steps, threads):
    """The CPU oracle (plain-C restatement of the reference, OpenMP over envs), timed on this host."""
    sys.path.insert(0, ROOT)
    from oracle import pyoracle as O
    threads = O.set_threads(threads)
    c = env.cfg_c
    init = env._init_states.cpu().numpy()
    rng = np.arange(2, dtype=np.uint32)
    keys = O.split_keys(rng[None], n_envs + 1)[0][1:]
    state, _ = O.env_reset(c, keys, init)
    t0 = time.perf_counter()
    master = np.array([0, 1], np.uint32)
    for _ in range(n_steps):
        ks = O.split_keys(master[None], n_envs + 1)[0]
        master, step_keys = ks[0].copy(), ks[1:].copy()
        acts = O.sample_actions(c, step_keys)
        state, *_ = O.env_step(c, step_keys, acts, day.msgs, init, state, with_info=False)
    dt = time.perf_counter() - t0
    return n_envs * n_steps / dt, threads


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=128)
    ap.add_argument("--warmup", type=int, default=16)
    ap.add_argument("--envs", type=int, default=NUM_ENVS, help="envs per GPU")
    ap.add_argument("--n-msgs", type=int, default=400_000, help="synthetic day length (messages)")
    ap.add_argument("--mid", type=int, default=2_000_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--graph-steps", type=int, default=0,
                    help="steps per captured HIP graph in the timed region (even; 0 = eager launches)")
    ap.add_argument("--config", default=CONFIG, help="builtin env config (the metric: 2_player_fq_fqc)")
    ap.add_argument("--mode", choices=("rollout", "step"), default="rollout",
                    help="rollout: one fused launch per step (key split + action sampling + step); "
                         "step: split_keys, sample_actions and env.step as three launches (SURVEY.md 8(d))")
    ap.add_argument("--slices", type=int, default=-1,
                    help="rollout mode: env slices on streams of their own (MARLEnv.rollout_sampled, 1..4; "
                         "-1 = MARLEnv.default_slices: 2 from 2048 envs up, else 1; 4 collapses on MI355X); "
                         "0 = one full-batch hftlob_env_step_sampled launch per step")
    ap.add_argument("--steps-per-call", type=int, default=0,
                    help="rollout mode with --slices: env steps per rollout_sampled call (0 = all timed steps)")
    ap.add_argument("--cpu-threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "16")))
    args = ap.parse_args()

    from hftlob import dist as D
    R = D.init_from_env("nccl")
    world, rank, local = R.world, R.rank, R.local
    torch.cuda.set_device(local)

    from hftlob.config_io import builtin_config
    from hftlob.data.synthetic import generate_day
    from hftlob.env import MARLEnv, split_keys
    from hftlob import _lib

    cfg = builtin_config(args.config)
    w = cfg.world_config
    snap = w.n_data_msg_per_step * w.start_resolution
    cache = f"/tmp/hftlob_day_{args.n_msgs}_{args.mid}_{snap}.npz"
    if rank == 0 and not os.path.exists(cache):
        d = generate_day(n_msgs=args.n_msgs, mid=args.mid, snap_every=snap)
        np.savez(cache + ".tmp.npz", msgs=d.msgs, books=d.books, snap_idx=d.snap_idx, tick=d.tick_size)
        os.replace(cache + ".tmp.npz", cache)
    D.barrier(R)
    from hftlob.data.synthetic import LobsterDay
    z = np.load(cache)
    day = LobsterDay(msgs=z["msgs"], books=z["books"], snap_idx=z["snap_idx"], tick_size=int(z["tick"]))

    E = args.envs
    env = MARLEnv(None, cfg, data=day, device=f"cuda:{local}", return_info=False, persistent_outputs=True)
    params = env.default_params
    # global key split, then this rank's slice (reference pmap layout: contiguous env blocks)
    master = torch.tensor([[0, 0]], dtype=torch.int32, device="cuda")
    all_keys = split_keys(master, world * E + 1)[0]
    keys0 = D.rank_keys(all_keys, rank, E).contiguous()
    _, state = env.reset(keys0, params)
    kbuf = [torch.tensor([0, 1 + rank], dtype=torch.int32, device="cuda"), torch.empty(2, dtype=torch.int32, device="cuda")]
    nstep = [0]

    rng = [kbuf[0].reshape(1, 2).clone()]

    if args.slices < 0:   # --graph-steps replays captured full-batch launches: unsliced
        args.slices = 0 if args.graph_steps > 0 else MARLEnv.default_slices(E)
    if args.graph_steps > 0 and args.slices > 0:
        raise SystemExit("--graph-steps needs --slices 0 (it captures full-batch launches)")
    sliced = args.mode == "rollout" and args.slices > 0
    T = (args.steps_per_call if args.steps_per_call > 0 else max(args.steps, 1)) if sliced else 1

    def one_step(n=1):
        k = nstep[0]
        if sliced:
            env.rollout_sampled(kbuf[k % 2], kbuf[(k + 1) % 2], state, params, n, n_slices=args.slices)
        elif args.mode == "rollout":
            env.step_sampled(kbuf[k % 2], kbuf[(k + 1) % 2], state, params)
        else:  # Speed_test's three calls, each its own launch: split, Discrete.sample, env.step
            ks = split_keys(rng[0], E + 1)[0]
            rng[0], sk = ks[0:1], ks[1:]
            env.step(sk, state, env.sample_actions(sk), params)
        nstep[0] = k + 1

    def run(n_steps):  # n_steps env steps as launches of T steps (the last one shorter)
        while n_steps > 0:
            one_step(min(T, n_steps))
            n_steps -= T

    run(args.warmup)
    torch.cuda.synchronize()
    G = (args.graph_steps if args.graph_steps > 0 and args.graph_steps % 2 == 0 and args.mode == "rollout"
         and T == 1 else 0)
    graph = None
    if G:
        # G consecutive launches in one HIP graph; G is even, so the key ping-pong buffers line up
        # between replays (every launch's pointers are baked in at capture)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            one_step()
            one_step()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            for _ in range(G):
                one_step()
        graph.replay()                        # one untimed replay (graph upload)
        torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    D.barrier(R)
    torch.cuda.synchronize()
    D.barrier(R)
    t0 = time.perf_counter()
    ev0.record()                              # on the launch stream (torch's current stream)
    done = 0
    if graph is not None:
        for _ in range(args.steps // G):
            graph.replay()
        done = args.steps // G * G
    run(args.steps - done)
    ev1.record()
    torch.cuda.synchronize()
    D.barrier(R)
    elapsed = time.perf_counter() - t0
    # HIP events on the launch stream bracket the timed region.  Full-batch launches: the
    # average k_env_step duration.  Sliced: per batched step (each k_env_step launch then
    # covers one slice; rocprof's per-launch average is ~the slice's share of it).
    kern_ms = ev0.elapsed_time(ev1) / args.steps
    # (step mode: the three launches of one step together; rocprof splits them)
    elapsed = D.max_over_ranks(R, elapsed, device="cuda")

    if rank != 0:
        D.finalize(R)
        return
    value = world * E * args.steps / elapsed
    per_env = algorithmic_bytes_per_env_step(env)
    achieved = per_env * E / (kern_ms * 1e-3) / 1e9
    traffic = None
    pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc):
        with open(pmc) as f:
            t = json.load(f)
        if t.get("hbm_bytes_per_env_step") is not None:   # per batched env step, like `achieved`
            traffic = round(t["hbm_bytes_per_env_step"] * E)
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        n_env_cpu, n_steps_cpu = 4096, 64       # one full episode (incl. auto-reset) of the metric workload
        v, thr = cpu_baseline(env, day, n_env_cpu, n_steps_cpu, args.cpu_threads)
        v1, _ = cpu_baseline(env, day, 512, 16, 1)
        cpu = {"value": round(v, 1), "unit": "env steps/s", "cores": thr, "kind": "port",
               "sample": f"{n_env_cpu} envs x {n_steps_cpu} steps of the same config/day, C oracle (OpenMP)",
               "single_core_value": round(v1, 1), "single_core_sample": "512 envs x 16 steps, 1 thread"}
    line = {
        "metric": "env steps/sec (whole node), 2-agent MARL, 10-level LOB, NUM_ENVS=4096",
        "value": round(value, 1),
        "unit": "env steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": f"synthetic LOBSTER day ({args.n_msgs} msgs, PCG64 seed 20260403, mid {args.mid})",
        "config": {"workload": (f"{CONFIG}.json MM fixed_quants + EXE fixed_quants_complex, 112 msgs/step, "
                                f"auto-reset, Speed_test semantics") if args.config == CONFIG else
                               f"{args.config}.json, {env.num_msgs_per_step} msgs/step, auto-reset, Speed_test semantics",
                   "num_envs_per_gpu": E, "num_envs_total": world * E, "parallelism": f"dp{world} (env shards)",
                   "launch": (f"hipGraph of {G} steps" if G else
                              (f"eager, {args.slices} env slices on their own streams (rollout_sampled, "
                               f"{T} steps per call)" if sliced else "eager")),
                   "mode": args.mode},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": round(achieved / PEAK_HBM_GBS, 5), "traffic": traffic,
                     "kernel": "k_env_step", "kernel_ms": round(kern_ms, 5), "slices": args.slices if sliced else 1,
                     "bytes_per_env_step": per_env},
        "cpu_baseline": cpu,
    }
    print(json.dumps(line))
    D.finalize(R)


if __name__ == "__main__":
    main()
