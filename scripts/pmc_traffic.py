"""HBM traffic per launch from a rocprofv3 PMC pass over bench.py
(scripts/pmc_bench.sh) -> profiles/pmc_<tag>.json, read by bench.py's
roofline `traffic` field.

bytes/launch = 2 * FETCH_SIZE + WRITE_SIZE (both reported in KiB), the gfx950
correction of MI355X_MICROARCH.md §HBM (FETCH_SIZE counts half the bytes of
streamed reads). That correction is calibrated for 16-byte lanes; the block's
kernels also read with 4-byte lanes, so the file carries a calibration row:
k_bn_stats reads each layer input exactly once (known byte count) with
4-byte loads.

Several pass directories (one per config) may be given: a kernel symbol
keeps the value of the first directory that has it (cfg2 first). A pass with
SQ_VALU_MFMA_BUSY_CYCLES and GRBM_GUI_ACTIVE adds `mfma_busy` per kernel: MFMA
busy cycles over the 1024 SIMDs x the kernel's cycles (GRBM_GUI_ACTIVE / 8 XCDs).

Round 3 on: one file per config, profiles/pmc_<tag>_<config>.json, carrying
"config" and "src_sha16" (bench.source_sha16() of the tree the passes ran on,
written by the GPU script into <pass dir>/../src_sha16.txt); bench.py only uses
the file of its config whose src_sha16 matches its own tree.

Usage: python scripts/pmc_traffic.py profiles/pmc_<tag>_<config>.json <pass dir> [...]
"""
import os
import csv
import glob
import json
import re
import sys
from collections import defaultdict

# bench.py cfg2 layer inputs (C_in, T) for N=128, V=18
LAYER_IN = [(3, 300), (64, 300), (64, 300), (64, 300), (64, 300), (128, 150), (128, 150),
            (128, 150), (256, 75), (256, 75)]


def short(name):
    m = re.search(r"stgcn::(\w+)(<[^>]*>)?", name)
    if not m:
        return None
    return m.group(1) + (m.group(2) or "").replace(" ", "")


def main(dst, *srcs):
    vals = defaultdict(lambda: defaultdict(list))
    for src in srcs:
        seen = defaultdict(lambda: defaultdict(list))
        for f in glob.glob(src + "/*/run_counter_collection.csv"):
            for r in csv.DictReader(open(f)):
                k = short(r.get("Kernel_Name", r.get("Kernel-Name", "")))
                if k:
                    seen[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, cs in seen.items():
            for c, v in cs.items():
                if c not in vals[k]:
                    vals[k][c] = v
    base = os.path.basename(dst)[:-5]  # pmc_<tag>_<config>
    tag, config = base.split("_")[1], base.split("_")[-1]
    sha = None
    for src in srcs:
        p = os.path.join(os.path.dirname(os.path.normpath(src)), "src_sha16.txt")
        if os.path.exists(p):
            sha = open(p).read().strip()
    out = {"tag": tag, "config": config, "src_sha16": sha,
           "source": f"rocprofv3 --pmc (separate passes) over bench.py --config {config} "
                     "--steps 2 --warmup 1 --no-roofline",
           "formula": "2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024 (bytes per launch)",
           "hbm_bytes_per_launch": {}, "raw_kib": {}, "mfma_busy": {}}
    for k, cs in sorted(vals.items()):
        if "FETCH_SIZE" not in cs or "WRITE_SIZE" not in cs:
            continue
        fs = sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"])
        ws = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"])
        out["hbm_bytes_per_launch"][k] = round(2 * fs * 1024 + ws * 1024)
        out["raw_kib"][k] = {"FETCH_SIZE": round(fs, 1), "WRITE_SIZE": round(ws, 1),
                             "launches": len(cs["FETCH_SIZE"])}
    for k, cs in sorted(vals.items()):
        if "SQ_VALU_MFMA_BUSY_CYCLES" in cs and "GRBM_GUI_ACTIVE" in cs:
            mb = sum(cs["SQ_VALU_MFMA_BUSY_CYCLES"]) / len(cs["SQ_VALU_MFMA_BUSY_CYCLES"])
            gg = sum(cs["GRBM_GUI_ACTIVE"]) / len(cs["GRBM_GUI_ACTIVE"]) / 8
            if gg > 0:
                out["mfma_busy"][k] = round(mb / (gg * 1024), 4)
    stats = [k for k in out["raw_kib"] if k.startswith("k_bn_stats")]
    if stats and config == "cfg2":
        # with stack chaining only block 0 runs its own BN1 statistics pass
        # (the other blocks take them from the previous block's output pass):
        # one launch per step reading the 3-channel input once
        alg = 128 * LAYER_IN[0][0] * LAYER_IN[0][1] * 18 * 4
        n = sum(out["raw_kib"][k]["launches"] for k in stats)
        fs = sum(out["raw_kib"][k]["FETCH_SIZE"] * out["raw_kib"][k]["launches"] for k in stats) * 1024 / n
        out["calibration_k_bn_stats"] = {
            "algorithmic_read_bytes": round(alg), "fetch_size_bytes": round(fs),
            "fetch_over_algorithmic": round(fs / alg, 3)}
    # bench.py keys its dominant kernel as k_tconv<9,2,V,1> (the same short names)
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out.get("calibration_k_bn_stats"), indent=1))
    for k, v in out["hbm_bytes_per_launch"].items():
        print(f"{k:40s} {v / 1e6:10.1f} MB/launch")


if __name__ == "__main__":
    main(sys.argv[1], *sys.argv[2:])
