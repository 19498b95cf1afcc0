"""GPU-busy vs wall time per training step from a rocprofv3 kernel trace of
bench.py (scripts/gpu_step_profile.sh): steps are delimited by the fused Adam
launch (one per step); busy = union of kernel intervals. A busy/wall ratio
near 1 means the step is not launch-bound (no host gaps for a hipGraph to
remove). Also prints the per-step time of the top kernels.

Usage: python scripts/step_busy.py gpurun_out/step_<tag>/run_kernel_trace.csv [steps]
"""
import csv
import sys
from collections import defaultdict


def main(path, steps=10):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    adam = [i for i, r in enumerate(rows) if "adam" in r["Kernel_Name"].lower()]
    seg = rows[adam[-steps - 1] + 1: adam[-1] + 1]
    t0, t1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["End_Timestamp"])
    busy, cs, ce = 0, None, None
    for r in seg:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if ce is None or s > ce:
            if ce is not None:
                busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    print(f"steps {steps}: wall {(t1 - t0) / 1e6 / steps:.3f} ms/step, GPU busy "
          f"{busy / 1e6 / steps:.3f} ms/step ({busy / (t1 - t0):.4f}), "
          f"{len(seg) / steps:.0f} launches/step")
    agg, cnt = defaultdict(float), defaultdict(int)
    for r in seg:
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
        k = name.split("(")[0][:90]
        agg[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 / steps
        cnt[k] += 1
    for k, v in sorted(agg.items(), key=lambda x: -x[1])[:40]:
        print(f"{v:8.3f} ms/step  {cnt[k] / steps:5.1f}x  {k}")
    # the last step's launches in order, with their durations
    last = rows[adam[-2] + 1: adam[-1] + 1]
    print("\nlast step, in launch order (us: duration, idle gap before the launch):")
    prev_end = None
    for r in last:
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:90]
        s0, e0 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s0 - prev_end) / 1e3 if prev_end is not None else 0.0
        prev_end = e0 if prev_end is None else max(prev_end, e0)
        print(f"{(e0 - s0) / 1e3:9.1f} {gap:7.1f}  {name}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 10)
