"""Average PMC counter values per kernel name across rocprofv3 passes."""
import csv
import glob
import sys
from collections import defaultdict

vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(sys.argv[1] + "/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", r.get("Kernel-Name", ""))
        vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
filt = sys.argv[2] if len(sys.argv) > 2 else ""
for k, cs in vals.items():
    if filt not in k:
        continue
    print(k[:80])
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {sum(v)/len(v):16.1f}  (n={len(v)})")
