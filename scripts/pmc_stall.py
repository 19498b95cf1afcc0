"""Stall breakdown per kernel from scripts/pmc_bench_k.sh / pmc_x3k.sh passes:
fractions of SQ_WAVE_CYCLES, MFMA busy per SIMD-cycle (SQ_VALU_MFMA_BUSY_CYCLES
over GRBM_GUI_ACTIVE/8 x 1024 SIMDs) and the clock.
Usage: python scripts/pmc_stall.py <dir-with-pass-subdirs> [name filter]"""
import csv
import glob
import sys
from collections import defaultdict

vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(sys.argv[1] + "/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", r.get("Kernel-Name", ""))
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
filt = sys.argv[2] if len(sys.argv) > 2 else ""
for k, cs in sorted(vals.items()):
    if filt not in k or "SQ_WAVE_CYCLES" not in cs:
        continue
    a = {c: sum(v) / len(v) for c, v in cs.items()}
    wc = a["SQ_WAVE_CYCLES"]
    gg = a.get("GRBM_GUI_ACTIVE", 0) / 8
    print(k[:90])
    print("   of wave cycles: wait_any %.3f wait_inst %.3f active %.3f | valu %.3f lds %.3f "
          "wait_lds %.3f vmem %.3f" % (a["SQ_WAIT_ANY"] / wc, a["SQ_WAIT_INST_ANY"] / wc,
                                       a["SQ_ACTIVE_INST_ANY"] / wc, a["SQ_ACTIVE_INST_VALU"] / wc,
                                       a["SQ_ACTIVE_INST_LDS"] / wc, a["SQ_WAIT_INST_LDS"] / wc,
                                       a.get("SQ_ACTIVE_INST_VMEM", 0) / wc))
    if gg:
        print("   mfma busy %.3f of SIMD cycles; kernel %.0f cycles; lds bank conflict / lds active %.3f"
              % (a["SQ_VALU_MFMA_BUSY_CYCLES"] / (gg * 1024), gg,
                 a.get("SQ_LDS_BANK_CONFLICT", 0) / max(1, a["SQ_ACTIVE_INST_LDS"])))
