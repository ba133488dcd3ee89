"""Print per-kernel average PMC counters from gpurun_out/<tag>_a and _b (tools/gpu_pmc.sh)."""
import csv
import glob
import sys
from collections import defaultdict

tag = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else ""
acc = defaultdict(lambda: defaultdict(list))
for part in ("a", "b"):
    for f in glob.glob(f"gpurun_out/{tag}_{part}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if kern in r["Kernel_Name"]:
                acc[r["Kernel_Name"][:50]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:24s} {sum(v) / len(v):16.1f}  (n={len(v)})")
