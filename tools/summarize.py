"""Summarise a GPU round: test tail, kernel stats of the rocprofv3 run, bench line."""
import csv
import json
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "x"
print(open("gpurun_out/gpu_tests.log").read().strip().split("\n")[-2:])
try:
    rows = list(csv.DictReader(open(f"gpurun_out/prof_{tag}/run_kernel_stats.csv")))
    for r in rows[:6]:
        print(f"{r['Name'][:80]:80s} {r['Calls']:>4} {float(r['AverageNs'])/1e3:10.1f} us {r['Percentage']}")
except FileNotFoundError:
    print("no profile")
b = json.loads(open("gpurun_out/bench.log").read().strip().split("\n")[-1])
print(b["value"], b["ms_per_step"], b["kernel_ms"], b["roofline"]["frac"], b.get("cpu_baseline", {}).get("value"))
