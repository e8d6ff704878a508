"""world_size-2 gloo run of the multi-GPU sharding logic on CPU (hftlob.dist,
used by bench.py): env blocks are disjoint and cover the global key split, and
the timing reduction is a max over ranks.  No collective touches env data."""
import os
import socket
import sys

import numpy as np
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, E, q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "jaxmarl-hft_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    from hftlob import dist as D
    from oracle import pyoracle as O
    r = D.init_from_env("gloo")
    all_keys = O.split_keys(np.array([[0, 0]], np.uint32), world * E + 1)[0]
    mine = D.rank_keys(all_keys, r.rank, E)
    gathered = [None] * world
    r.dist.all_gather_object(gathered, (r.rank, mine.tolist()))
    t = D.max_over_ranks(r, 1.5 + r.rank)
    D.barrier(r)
    if r.rank == 0:
        q.put((gathered, t, all_keys.tolist()))
    D.finalize(r)


def test_two_rank_sharding():
    world, E = 2, 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(i, world, port, E, q)) for i in range(world)]
    for p in procs:
        p.start()
    gathered, t, all_keys = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    gathered.sort()
    union = [k for _, ks in gathered for k in ks]
    assert union == all_keys[1:]                     # disjoint, contiguous, covering
    assert len({tuple(k) for k in union}) == world * E
    assert t == 2.5                                  # max over ranks
