"""Summarise a tools/profile_round.sh directory: kernel stats, HBM traffic per
env-step (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE), SQ counters per env-step.
Writes <dir>/pmc_traffic.json and <dir>/kernel_profile.json (what bench.py reads from
profiles/rNN_kernel_profile.json for the roofline's traffic and the issue roofline) and
prints a text summary.

The metric kernel is k_env_step (env slices: one launch = one step of E / G envs, G launches
in flight) or k_env_rollout (the persistent launch: every wave runs its env's steps back to
back; per-wave counters are divided by the steps per launch, `steps_per_launch` in
<dir>/shape.json, written by profile_round.sh)."""
import csv
import glob
import json
import os
import sys

d = sys.argv[1]


def rows(sub, pat="*counter_collection.csv"):
    f = glob.glob(os.path.join(d, sub, "**", pat), recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


shape = json.load(open(os.path.join(d, "shape.json"))) if os.path.exists(os.path.join(d, "shape.json")) else {}
KERNEL = shape.get("kernel", "k_env_step")
SPL = shape.get("steps_per_launch", 1)        # PMC passes: env-steps per wave per launch
STATS_SPL = shape.get("stats_steps_per_launch", 1)  # the stats run: steps per launch


def per_launch(sub, counter, kernel=KERNEL):
    vals = [float(r["Counter_Value"]) for r in rows(sub) if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter]
    return sum(vals) / len(vals) if vals else None


stats = glob.glob(os.path.join(d, "stats", "**", "*kernel_stats.csv"), recursive=True)
kstat = None
if stats:
    print("== rocprofv3 --kernel-trace --stats (bench.py --no-cpu-baseline)")
    for r in csv.DictReader(open(stats[0])):
        print(f"{r['Name'][:60]:60s} calls {r['Calls']:>6s} avg_ns {float(r['AverageNs']):12.1f} "
              f"total_pct {float(r['Percentage']):6.2f}")
        if KERNEL in r["Name"] and kstat is None:
            kstat = {"kernel_avg_us": round(float(r["AverageNs"]) / 1e3, 2), "launches": int(r["Calls"]),
                     "kernel_name": r["Name"], "steps_per_launch": STATS_SPL,
                     "kernel_us_per_step": round(float(r["AverageNs"]) / 1e3 / STATS_SPL, 3)}
stats20 = glob.glob(os.path.join(d, "stats20", "**", "*kernel_stats.csv"), recursive=True)
kstat20 = None
for r in (csv.DictReader(open(stats20[0])) if stats20 else []):
    if KERNEL in r["Name"]:  # two 20-step launches (--warmup 20 --steps 20): the driver's launch length
        kstat20 = {"kernel_avg_us": round(float(r["AverageNs"]) / 1e3, 2), "launches": int(r["Calls"]),
                   "steps_per_launch": 20, "kernel_us_per_step": round(float(r["AverageNs"]) / 1e3 / 20, 3)}
        print("== rocprofv3 stats, 20-step launches:", kstat20)
        break
fetch_kb, write_kb = per_launch("fetch", "FETCH_SIZE"), per_launch("write", "WRITE_SIZE")
bench = json.load(open(os.path.join(d, "stats_bench.json"))) if os.path.exists(os.path.join(d, "stats_bench.json")) else {}
E = bench.get("config", {}).get("num_envs_per_gpu", 4096)
G = shape.get("slices", bench.get("roofline", {}).get("launches_per_step", 1)) or 1
# env slices: one k_env_step launch steps E / G envs; the persistent launch steps all E envs SPL times
out = {}
if fetch_kb is not None and write_kb is not None:
    hbm = (2 * fetch_kb + write_kb) * 1024
    out = {"kernel": KERNEL, "fetch_size_kb_raw": fetch_kb, "write_size_kb": write_kb,
           "correction": "FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md HBM section)",
           "hbm_bytes_per_launch": round(hbm), "hbm_bytes_per_env_step": round(hbm * G / E / SPL, 1),
           "envs_per_launch": E // G, "steps_per_launch": SPL}
    json.dump(out, open(os.path.join(d, "pmc_traffic.json"), "w"), indent=1)
    print(f"== HBM traffic per {KERNEL} launch:", json.dumps(out))
fetch20, write20 = per_launch("fetch20", "FETCH_SIZE"), per_launch("write20", "WRITE_SIZE")
if out and fetch20 is not None and write20 is not None:  # the driver's shape: one 20-step launch
    out["hbm_bytes_per_env_step_20_step_launch"] = round((2 * fetch20 + write20) * 1024 / E / 20, 1)
    json.dump(out, open(os.path.join(d, "pmc_traffic.json"), "w"), indent=1)
    print("== HBM traffic per env-step, one 20-step launch:", out["hbm_bytes_per_env_step_20_step_launch"])
sq = {}
for r in rows("sq"):
    if KERNEL in r["Kernel_Name"]:
        sq.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
per_wave = {}
if sq:
    w = sum(sq["SQ_WAVES"]) / len(sq["SQ_WAVES"])
    per_wave = {k.replace("SQ_", ""): round(sum(v) / len(v) / w / SPL, 1) for k, v in sorted(sq.items())
                if k != "SQ_WAVES"}
    print(f"== SQ counters per wave and env-step ({KERNEL}):", per_wave)
sq20 = {}
for r in rows("sq20"):  # the driver's launch length: one 20-step launch
    if KERNEL in r["Kernel_Name"]:
        sq20.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
per_wave20 = {}
if sq20:
    w = sum(sq20["SQ_WAVES"]) / len(sq20["SQ_WAVES"])
    per_wave20 = {k.replace("SQ_", ""): round(sum(v) / len(v) / w / 20, 1) for k, v in sorted(sq20.items())
                  if k != "SQ_WAVES"}
    print(f"== SQ counters per wave and env-step, one 20-step launch ({KERNEL}):", per_wave20)
lds = {}
for r in rows("lds"):
    if KERNEL in r["Kernel_Name"]:
        lds.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
if lds:
    w = sum(lds["SQ_WAVES"]) / len(lds["SQ_WAVES"])
    print(f"== SQ LDS / issue counters per wave and env-step ({KERNEL}):",
          {k.replace("SQ_", ""): round(sum(v) / len(v) / w / SPL, 1) for k, v in sorted(lds.items()) if k != "SQ_WAVES"})
sm = os.path.join(d, "bench_stepmode.json")
if os.path.exists(sm) and os.path.getsize(sm):
    b = json.load(open(sm))
    print("== step mode (split_keys + sample_actions + env.step, 3 launches):", b["value"], "env steps/s,",
          b["ms_per_step"], "ms/step")

# one wave per env: per-wave counts / steps per launch are per env-step
prof = dict(kstat or {})
if kstat20:
    prof["rocprof_20_step_launch"] = kstat20
prof.update({"kernel": KERNEL, "slices": shape.get("slices", G), "envs_per_launch": E // G,
             "launches_in_flight": G, "source": os.path.basename(os.path.normpath(d)),
             "commit": shape.get("commit") or os.environ.get("PROF_COMMIT")})
if "INSTS_SALU" in per_wave20:
    prof["salu_per_env_step_by_launch_steps"] = {str(SPL): per_wave.get("INSTS_SALU"), "20": per_wave20["INSTS_SALU"]}
if "INSTS_SALU" in per_wave:
    prof["salu_per_env_step"] = per_wave["INSTS_SALU"]
    prof["valu_per_env_step"] = per_wave.get("INSTS_VALU")
    prof["wave_cycles_per_env_step"] = per_wave.get("WAVE_CYCLES")
if out:  # keyed by the launch length the traffic was counted on
    prof["hbm_bytes_per_env_step"] = out["hbm_bytes_per_env_step"]
    prof["traffic_steps_per_launch"] = SPL
    prof["hbm_bytes_per_env_step_by_launch_steps"] = {str(SPL): out["hbm_bytes_per_env_step"]}
    if "hbm_bytes_per_env_step_20_step_launch" in out:
        prof["hbm_bytes_per_env_step_by_launch_steps"]["20"] = out["hbm_bytes_per_env_step_20_step_launch"]
json.dump(prof, open(os.path.join(d, "kernel_profile.json"), "w"), indent=1)
print("== kernel_profile.json:", json.dumps(prof))
