"""Per-loop instruction counts of one kernel's ISA (hipcc -S output): every basic block is
assigned to its innermost loop from the compiler's "Loop Header" / "in Loop: Header=" comments,
and each loop (with its child loops) gets counts of SGPR spill reloads / stores (v_readlane /
v_writelane on the spill VGPRs), scratch accesses, SALU / VALU / LDS / branch instructions.
Usage: python tools/isa_loops.py FILE.s KERNEL_SUBSTRING"""
import re
import sys
from collections import defaultdict


def main(path, kname):
    lines = open(path).read().split("\n")
    start = next(i for i, ln in enumerate(lines) if ln.startswith("_Z") and kname in ln and ln.rstrip().endswith(":") or
                 (ln.startswith("_Z") and kname in ln and ": ;" in ln))
    end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
    body = lines[start:end + 1]
    spill_v = set()
    for ln in body:
        m = re.search(r"v_writelane_b32 (v\d+), s\d+, \d+$", ln.strip())
        if m:
            if int(m.group(1)[1:]) >= 120 and ln.strip().endswith(tuple(str(k) for k in range(64))):
                spill_v.add(m.group(1))
    # loop membership: block -> innermost header; header -> parent
    parent, cur, counts = {}, None, defaultdict(lambda: defaultdict(int))
    for ln in body:
        m = re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):", ln)
        if m:
            name = m.group(1).replace("; %bb.", ".LBB0_")
            h = re.search(r"Header=BB(\d+_\d+)", ln)
            if "This Loop Header" in ln or "=>" in ln:
                cur = name.lstrip(".").replace("LBB", "BB")
            elif h:
                cur = "BB" + h.group(1)
            else:
                cur = None
            continue
        mp = re.search(r"Parent Loop BB(\d+_\d+)", ln)
        if mp and cur:
            parent.setdefault(cur, set()).add("BB" + mp.group(1))
        s = ln.strip()
        if not s or s.startswith(";") or s.startswith("."):
            continue
        op = s.split()[0]
        c = counts[cur]
        c["insts"] += 1
        if op == "v_readlane_b32" and s.split(",")[1].strip() in spill_v:
            c["sgpr_reload"] += 1
        if op == "v_writelane_b32" and s.split()[1].rstrip(",") in spill_v:
            c["sgpr_spill"] += 1
        if op.startswith("scratch_"):
            c["scratch"] += 1
        if op.startswith("s_cbranch") or op == "s_branch":
            c["branch"] += 1
        elif op.startswith("s_waitcnt"):
            c["waitcnt"] += 1
        elif op.startswith("s_load") or op.startswith("s_buffer_load"):
            c["smem"] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
        elif op.startswith("v_"):
            c["valu"] += 1
        elif op.startswith("ds_"):
            c["lds"] += 1
        elif op.startswith("global_") or op.startswith("flat_") or op.startswith("buffer_"):
            c["vmem"] += 1
    print(f"spill VGPRs: {sorted(spill_v)}")
    keys = ["insts", "salu", "valu", "lds", "smem", "vmem", "branch", "sgpr_reload", "sgpr_spill", "scratch"]
    print("loop".ljust(12) + "".join(k.rjust(12) for k in keys))
    for h in sorted(counts, key=lambda x: (x is None, x or "")):
        c = counts[h]
        print(str(h).ljust(12) + "".join(str(c[k]).rjust(12) for k in keys))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
