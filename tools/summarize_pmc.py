"""Sum rocprofv3 --pmc counter_collection CSVs per kernel (all passes under a dir)."""
import csv, glob, os, sys
from collections import defaultdict
root = sys.argv[1]
tot = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for f in glob.glob(os.path.join(root, "**", "*counter_collection*.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "?")[:60]
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add((f, r.get("Dispatch_Id")))
for k, c in tot.items():
    if not any("batch" in k or "sparse" in k or "minplus" in k for _ in [0]):
        continue
    print(k)
    for name in sorted(c):
        print(f"   {name:28s} {c[name]:.4g}")
