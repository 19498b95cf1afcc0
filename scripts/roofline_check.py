"""Recompute a bench line's roofline fraction from the rocprofv3 kernel summary
of the same command (each config's roofline.frac must be
recomputable as algorithmic work / the rocprof average of the named kernel /
peak).

The bench line names the dominant kernel by its rocprof short name and carries
its algorithmic FLOPs and bytes per launch; the kernel_stats.csv of the
`rocprofv3 --kernel-trace --stats` run of the same bench command gives the
average duration of every launch of that symbol (the bench's own timing
launches included: they use the block's launch parameters).

Usage: python scripts/roofline_check.py <bench.json> <kernel_stats.csv> [out.json]
"""
import csv
import json
import re
import sys


def short(name):
    m = re.search(r"stgcn::(\w+)(<[^>]*>)?", name)
    if not m:
        return None
    return m.group(1) + (m.group(2) or "").replace(" ", "")


def main(bench_path, stats_path, out_path=None):
    line = json.load(open(bench_path))
    r = line["roofline"]
    sym = r["kernel"]
    # bench names a few kernels as families (k_conv_x3<5|4,...>): match each member
    pats = [sym]
    if "<5|4," in sym:
        pats = [sym.replace("<5|4,", "<5,5,"), sym.replace("<5|4,", "<4,4,")]
    rows = [x for x in csv.DictReader(open(stats_path)) if short(x["Name"]) in pats]
    if not rows:
        raise SystemExit(f"{sym}: not in {stats_path}")
    calls = sum(int(x["Calls"]) for x in rows)
    tot_ns = sum(float(x["TotalDurationNs"]) for x in rows)
    avg_ms = tot_ns / calls / 1e6
    if r["bound"] == "mfma":
        work = r["algorithmic_flops_per_launch"] / 1e12  # TFLOP
    else:
        work = r["algorithmic_bytes_per_launch"] / 1e9   # GB
    ach = work / (avg_ms * 1e-3)
    out = {"config": line["config"]["workload"][:4], "kernel": sym, "bound": r["bound"],
           "bench_avg_launch_ms": r["avg_launch_ms"], "rocprof_avg_ms": round(avg_ms, 4),
           "rocprof_calls": calls, "unit": r["unit"], "peak": r["peak"],
           "achieved_rocprof": round(ach, 2), "frac_rocprof": round(ach / r["peak"], 4),
           "frac_bench": r["frac"],
           "agree": abs(avg_ms - r["avg_launch_ms"]) / r["avg_launch_ms"] < 0.10}
    print(json.dumps(out))
    if out_path:
        json.dump(out, open(out_path, "w"), indent=1)
    return out


if __name__ == "__main__":
    main(*sys.argv[1:])
