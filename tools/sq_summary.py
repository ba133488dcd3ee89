#!/usr/bin/env python3
"""Summarise tools/gpu_sq_profile.sh output: per program and kernel, the mean per-dispatch counter values and the
derived shares (VALU / LDS busy, LDS bank-conflict share, waits).  Usage: sq_summary.py TAG > profiles/<...>.md
Units (MI355X_MICROARCH.md): SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles summed over waves;
SQ_BUSY_CYCLES counts cycles the SQs were busy (summed over SEs/XCDs); GRBM_GUI_ACTIVE is summed over the 8 XCDs."""
import csv
import glob
import sys
from collections import defaultdict

tag = sys.argv[1]


def kname(full):
    """The engine's kernels only (input synthesis and fills are not part of the path)."""
    if "sdrg" not in full:
        return None
    return full.replace("void ", "").replace("sdrg::(anonymous namespace)::", "").replace("sdrg::", "").split("(")[0][:70]
progs = {"spec": "spectrum alone (4096 x 16384 CS8, 10 calls)", "c2": "spectrum + stats (4096 x 16384, 5 kHz)",
         "c5": "spectrum + stats (1024 x 65536 CS16, 200 kHz)", "c3": "all stages pipelined (the c3 step, co-resident)",
         "ssb": "SSB stage alone (4096 x 16384 CS8, 10 calls)"}
print(f"# SQ counters ({tag}): rocprofv3 --kernel-trace --pmc, one pass per group (tools/gpu_sq_profile.sh)\n")
for p, desc in progs.items():
    acc = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for part in "abc":
        for f in glob.glob(f"gpurun_out/{tag}_{p}_{part}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                k = kname(r["Kernel_Name"])
                if k is None:
                    continue
                acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for f in glob.glob(f"gpurun_out/{tag}_{p}_{part}/**/*kernel_trace.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                k = kname(r["Kernel_Name"])
                if k is None:
                    continue
                dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    if not acc:
        continue
    print(f"## {p}: {desc}\n")
    for k, d in sorted(acc.items(), key=lambda kv: -sum(dur.get(kv[0], [0]))):
        m = {c: sum(v) / len(v) for c, v in d.items()}
        us = sorted(dur.get(k, [0]))
        med = us[len(us) // 2] if us else 0
        print(f"### `{k}` — median dispatch {med:.1f} us (profiled passes)\n")
        print("| counter | per dispatch |\n|---|---|")
        for c in sorted(m):
            print(f"| {c} | {m[c]:.4g} |")
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            print()
            for c in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY",
                      "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VMEM"):
                if c in m:
                    print(f"- {c} / SQ_WAVE_CYCLES = {m[c] / wc:.3f}")
        if m.get("SQ_LDS_IDX_ACTIVE"):
            print(f"- SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE = {m.get('SQ_LDS_BANK_CONFLICT', 0) / m['SQ_LDS_IDX_ACTIVE']:.3f}")
        if m.get("SQ_WAVES"):
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"):
                if c in m:
                    print(f"- {c} per wave = {m[c] / m['SQ_WAVES']:.1f}")
        if m.get("GRBM_GUI_ACTIVE") and med:
            print(f"- effective clock GRBM_GUI_ACTIVE / 8 / duration = {m['GRBM_GUI_ACTIVE'] / 8 / (med * 1e3):.3f} GHz")
        print()
