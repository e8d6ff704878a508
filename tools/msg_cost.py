"""Per-message-kind instruction cost of the engine (k_book_process<2>).

GPU mode (run under rocprofv3 --pmc ...): builds a 40+40-order book, then
runs one dispatch per message kind over 4096 envs x 448 messages, in the
order of KINDS (after a warm-up dispatch).  Report mode (--report DIR) reads
the rocprofv3 counter CSV and prints SQ counters per message per wave.
"""
import csv
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "jaxmarl-hft_amd")]

import numpy as np  # noqa: E402

KINDS = ["noop", "cancel_partial", "add_then_delete", "add_then_cross", "exec_ioc", "mixed_random", "full_add",
         "cancel_wrap"]
FULL = ("full_add", "cancel_wrap")  # run on a book whose sides hold 100 orders each (every add evicts)
E, N = 4096, 448


def stream(kind, rng):
    m = np.zeros((N, 8), np.int32)
    t = 34300
    for k in range(N):
        tn = 1000 + k
        s = 1 if k % 2 == 0 else -1
        if kind == "noop":
            row = (0, 0, 0, 0, 0, 0, t, tn)
        elif kind == "cancel_partial":
            j = (k // 2) % 40
            row = (2, s, 1, (990 - j) if s == 1 else (1010 + j), (1 + j) if s == 1 else (101 + j), 7, t, tn)
        elif kind == "add_then_delete":
            j = k // 2
            row = (1, 1, 5, 980, 5000 + j, 7, t, tn) if k % 2 == 0 else (3, 1, 5, 980, 5000 + j, 7, t, tn)
        elif kind == "add_then_cross":
            j = k // 2
            row = (1, -1, 5, 1005, 5000 + j, 7, t, tn) if k % 2 == 0 else (1, 1, 5, 1005, 9000 + j, 8, t, tn)
        elif kind == "exec_ioc":
            row = (4, s, 1, 990 if s == 1 else 1010, 0, 7, t, tn)   # executes the touch (side flipped)
        elif kind == "full_add":  # a limit order into a full side: check_book_fill evicts the worst level
            p = (985 - int(rng.integers(0, 60))) if s == 1 else (1015 + int(rng.integers(0, 60)))
            row = (1, s, int(rng.integers(1, 50)), p, 30000 + k, 7, t, tn)
        elif kind == "cancel_wrap":  # an id no row holds, no init-id row at its price: the -1 index wraps to
            p = 500 if s == 1 else 1500  # the last slot, which holds an order (partial cancel of it)
            row = (2, s, 1, p, 70000 + k, 7, t, tn)
        else:
            u = rng.random()
            if u < 0.45:
                p = (990 - int(rng.integers(0, 10))) if s == 1 else (1010 + int(rng.integers(0, 10)))
                row = (1, s, int(rng.integers(1, 50)), p, 20000 + k, 7, t, tn)
            elif u < 0.9:
                j = int(rng.integers(0, 40))
                row = (2, s, 1, (990 - j) if s == 1 else (1010 + j), (1 + j) if s == 1 else (101 + j), 7, t, tn)
            else:
                row = (4, s, 1, 990 if s == 1 else 1010, 0, 7, t, tn)
        m[k] = row
    return m


def run():
    import torch
    from hftlob.config_io import builtin_config
    from hftlob.engine import book_process_
    w = builtin_config("2_player_fq_fqc").world_config
    dev = "cuda"
    init = np.zeros((80, 8), np.int32)
    for j in range(40):
        init[2 * j] = (1, 1, 1000, 990 - j, 1 + j, 3, 34200, j)
        init[2 * j + 1] = (1, -1, 1000, 1010 + j, 101 + j, 3, 34200, j)
    asks = torch.full((E, w.nOrders, 6), -1, dtype=torch.int32, device=dev)
    bids, trades = torch.full_like(asks, -1), torch.full((E, w.nTrades, 8), -1, dtype=torch.int32, device=dev)
    book_process_(w, torch.from_numpy(np.broadcast_to(init, (E, 80, 8)).copy()).to(dev), asks, bids, trades)
    rng = np.random.default_rng(3)
    # the full book: 60 more orders per side, behind the 40 levels of the base book
    fill = np.zeros((120, 8), np.int32)
    for j in range(60):
        fill[2 * j] = (1, 1, 1000, 940 - j, 201 + j, 3, 34200, 100 + j)
        fill[2 * j + 1] = (1, -1, 1000, 1060 + j, 301 + j, 3, 34200, 100 + j)
    fa, fb, ft = asks.clone(), bids.clone(), trades.clone()
    book_process_(w, torch.from_numpy(np.broadcast_to(fill, (E, 120, 8)).copy()).to(dev), fa, fb, ft)
    for kind in ["noop"] + KINDS:
        msgs = torch.from_numpy(np.broadcast_to(stream(kind, rng), (E, N, 8)).copy()).to(dev)
        a, b, t = (fa.clone(), fb.clone(), ft.clone()) if kind in FULL else (asks.clone(), bids.clone(), trades.clone())
        ba = torch.empty((E, N, 2), dtype=torch.int32, device=dev)
        bb = torch.empty_like(ba)
        book_process_(w, msgs, a, b, t, ba, bb)
    torch.cuda.synchronize()


def report(d):
    import glob
    disp = collections.OrderedDict()
    for f in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
        rows = [r for r in csv.DictReader(open(f))
                if "k_book_process" in r["Kernel_Name"] and int(r["Grid_Size"]) == E * 64]
        ids = sorted({int(r["Dispatch_Id"]) for r in rows})[-len(KINDS):]
        for r in rows:
            i = int(r["Dispatch_Id"])
            if i in ids:
                disp.setdefault(KINDS[ids.index(i)], {})[r["Counter_Name"]] = float(r["Counter_Value"])
    names = sorted({k for v in disp.values() for k in v} - {"SQ_WAVES"})
    short = [n.replace("SQ_", "").replace("INSTS_", "I_").replace("ACTIVE_INST_", "A_").replace("ICACHE_", "IC_")
             for n in names]
    # wall time per message of each dispatch (kernel trace of the same runs), 4096 envs in flight
    dur = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)):
        rows = [r for r in csv.DictReader(open(f))
                if "k_book_process" in r["Kernel_Name"] and int(r.get("Grid_Size_X") or r.get("Grid_Size")) == E * 64]
        rows.sort(key=lambda r: int(r["Dispatch_Id"]))
        for kind, r in zip(KINDS, rows[-len(KINDS):]):
            dur[kind].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / N)
    if dur:
        print("ns per message (whole batch of 4096 envs, min over passes):")
        for kind in KINDS:
            print(f"  {kind:18s} {min(dur[kind]):8.1f}")
    print("per message per wave (cycle counters in quad-cycles; SQC_* per message per CU-pair estimate):")
    print(f"{'':18s}" + "".join(f"{s:>10s}" for s in short))
    for kind in KINDS:
        v = disp.get(kind, {})
        print(f"{kind:18s}" + "".join(f"{v.get(n, float('nan')) / E / N:10.1f}" for n in names))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--report":
        report(sys.argv[2])
    else:
        run()
