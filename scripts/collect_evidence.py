"""Copy one gpu_evidence_r3.sh call's results (gpurun_out/ev_<tag>/) into
profiles/: the bench lines, the rocprofv3 kernel summaries (csv + a text top
list), the per-step kernel breakdown of the config's first timed run, and the
GPU pytest log tail.

Usage: python scripts/collect_evidence.py <tag> [cfg ...]
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def top_text(path, n=30):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    out = []
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
        out.append(f"{float(r['TotalDurationNs'])/1e6:9.2f} ms {float(r['Percentage']):6.2f}% "
                   f"calls={r['Calls']:>5} avg={float(r['AverageNs'])/1e3:9.1f}us  {r['Name'][:90]}")
    out.append(f"total {tot/1e6:.2f} ms")
    return "\n".join(out) + "\n"


def step_text(trace, steps=10, skip=3):
    """Per-step kernel time over the FIRST `steps` Adam-delimited steps after
    the warmup of the first timed run (the bench's default path; cfg2 runs its
    exact fp32-MFMA alternative afterwards)."""
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    # one Adam update per step (the device-step form also launches its counter
    # tick, k_adam_tick, which is not counted as a step boundary)
    adam = [i for i, r in enumerate(rows)
            if "adam" in r["Kernel_Name"].lower() and "tick" not in r["Kernel_Name"]]
    # bench: W warmup steps then K timed steps per run; the warmup is 3 in the
    # evidence script (in the HIP-graph mode: eager steps + untimed replays), so the
    # first timed step starts after the skip-th Adam
    seg = rows[adam[skip - 1] + 1: adam[skip - 1 + steps] + 1]
    t0, t1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["End_Timestamp"])
    per = {}
    for r in seg:
        per[r["Kernel_Name"]] = per.get(r["Kernel_Name"], 0) + \
            int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    busy = sum(per.values())
    lines = [f"steps {steps} (first timed run): wall {(t1 - t0) / 1e6 / steps:.3f} ms/step, "
             f"kernel time {busy / 1e6 / steps:.3f} ms/step, {len(seg) // steps} launches/step"]
    for k, v in sorted(per.items(), key=lambda kv: -kv[1])[:30]:
        lines.append(f"  {v / 1e6 / steps:7.3f} ms/step  {k.split('(')[0][:80]}")
    return "\n".join(lines) + "\n"


def main(tag, cfgs):
    src = os.path.join(ROOT, "gpurun_out", f"ev_{tag}")
    dst = os.path.join(ROOT, "profiles")
    for c in cfgs:
        b = os.path.join(src, f"bench_{c}.json")
        if os.path.exists(b):
            d = json.load(open(b))
            json.dump(d, open(os.path.join(dst, f"{tag}_bench_{c}.json"), "w"), indent=1)
            print(c, d["value"], d.get("roofline", {}).get("kernel"), d.get("roofline", {}).get("frac"))
        st = os.path.join(src, f"stats_{c}", "run_kernel_stats.csv")
        if os.path.exists(st):
            shutil.copy(st, os.path.join(dst, f"{tag}_kernel_stats_{c}.csv"))
            open(os.path.join(dst, f"{tag}_kernel_stats_{c}.txt"), "w").write(top_text(st))
        tr = os.path.join(src, f"stats_{c}", "run_kernel_trace.csv")
        if os.path.exists(tr):
            # (W = 3 warm-up steps in either step mode: eager, or 2 eager + the
            # capture + 1 untimed replay; r6x ran 3 eager + 1 replay: skip 4)
            sb = os.path.join(src, f"stats_bench_{c}.json")
            graph = os.path.exists(sb) and json.load(open(sb)).get("step_mode") == "hip_graph"
            skip = 4 if graph and tag == "r6x" else 3
            open(os.path.join(dst, f"{tag}_step_{c}.txt"), "w").write(step_text(tr, skip=skip))
    lg = os.path.join(src, "pytest_gpu.log")
    if os.path.exists(lg):
        lines = open(lg).read().splitlines()
        keep = [l for l in lines if "PASSED" in l or "FAILED" in l or "SKIPPED" in l or "ERROR" in l]
        open(os.path.join(dst, f"{tag}_pytest_gpu.txt"), "w").write(
            "\n".join(keep + lines[-2:]) + "\n")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:] or ["cfg2", "cfg3", "cfg5"])
