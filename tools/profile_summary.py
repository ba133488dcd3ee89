"""Summarise tools/profile_round.sh output into profiles/ (committed evidence for the bench line).

    python tools/profile_summary.py TAG

Writes profiles/TAG_kernel_stats.csv (rocprofv3 --stats, as produced), profiles/TAG_bench.json (the bench
line), profiles/TAG_hbm_pmc.json (FETCH_SIZE / WRITE_SIZE per launch of each engine kernel, with the
gfx950 correction of MI355X_MICROARCH.md: FETCH_SIZE counts half the bytes of wide coalesced reads, so it is
doubled; rocprofv3 reports both in KiB) and profiles/TAG_summary.md.
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

TAG = sys.argv[1] if len(sys.argv) > 1 else "r1"
OUT = "profiles"
os.makedirs(OUT, exist_ok=True)
ENGINE = ("spectrum16k_kernel", "spectrum_kernel", "stats_narrow_kernel", "stats_wide_multi_kernel", "stats_wide_kernel", "stats_kernel", "ssb_pipe_kernel", "four_step_a", "four_step_b", "ssb_chain_kernel",
          "ssb_fir_kernel", "ssb_eq_kernel", "spectral_pulse_kernel", "audio_pulse_kernel", "audio_front_kernel",
          "pulse_reset_kernel")


def short(name: str) -> str:
    for k in ENGINE:
        if k in name:
            return k
    return name[:60]


def counters(path: str, counter: str):
    per = defaultdict(list)
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                per[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return per


stats_csv = glob.glob(f"gpurun_out/prof_{TAG}/**/*kernel_stats.csv", recursive=True)
lines = [f"# Round profile {TAG}", ""]
if stats_csv:
    shutil.copy(stats_csv[0], f"{OUT}/{TAG}_kernel_stats.csv")
    lines += ["## rocprofv3 --kernel-trace --stats (bench.py --steps 40 --warmup 50 --no-cpu-baseline, defaults)", "",
              "| kernel | calls | avg us | min us | max us | % |", "|---|---|---|---|---|---|"]
    for r in csv.DictReader(open(stats_csv[0])):
        lines.append(f"| {short(r['Name'])} | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
                     f"{float(r['MinNs']) / 1e3:.1f} | {float(r['MaxNs']) / 1e3:.1f} | {r['Percentage']} |")
# per-launch durations of the roofline kernel from the trace, split by whether the launch overlapped an SSB
# pipeline launch (the pipelined schedule: co-resident) or ran with no SSB work on the chip (the isolated leg
# and the FFT + statistics labelled leg)
trace_csv = glob.glob(f"gpurun_out/prof_{TAG}/**/*kernel_trace.csv", recursive=True)
if trace_csv:
    allr = list(csv.DictReader(open(trace_csv[0])))
    iv = lambda r: (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
    ssb = [iv(r) for r in allr if "ssb_pipe_kernel" in r["Kernel_Name"]]
    co, alone = [], []
    for r in allr:
        if "spectrum16k_kernel" not in r["Kernel_Name"]:
            continue
        s0, e0 = iv(r)
        (co if any(s < e0 and s0 < e for s, e in ssb) else alone).append((e0 - s0) / 1e3)
    if co and alone:
        lines += ["", "## spectrum16k_kernel launch durations from the kernel trace", "",
                  f"* beside an SSB pipeline launch ({len(co)} launches, the pipelined schedule): "
                  f"avg {sum(co) / len(co):.1f} us",
                  f"* with no SSB work on the chip ({len(alone)} launches: the isolated leg and the FFT + statistics "
                  f"labelled leg): avg {sum(alone) / len(alone):.1f} us",
                  "* the bench line's `roofline` / `roofline_isolated` time the same two situations with HIP events"]
    # the SSB stream per step in the pipelined schedule: consecutive ssb_pipe_kernel launches that overlap a spectrum launch,
    # start to start (the pipeline kernel + the audio pulse detector + launch gaps), against the profiled run's own line
    spec = [iv(r) for r in allr if "spectrum16k_kernel" in r["Kernel_Name"]]
    ssb_s = sorted(ssb)
    cad = []
    for (a0, a1), (b0, b1) in zip(ssb_s, ssb_s[1:]):
        if any(s < a1 and a0 < e for s, e in spec) and any(s < b1 and b0 < e for s, e in spec) and b0 - a0 < 1_000_000:
            cad.append((b0 - a0) / 1e6)
    dur = [(e - s) / 1e6 for s, e in ssb_s]
    prof_line = None
    plog = f"gpurun_out/prof_bench_{TAG}.log"
    if os.path.exists(plog):
        for ln in open(plog):
            if ln.startswith("{"):
                prof_line = json.loads(ln)
    if cad:
        cad.sort()
        med = cad[len(cad) // 2]
        lines += ["", "## SSB stream per step (pipelined schedule) from the kernel trace", "",
                  f"* ssb_pipe_kernel start to next start, both beside a spectrum launch: median {med:.4f} ms over "
                  f"{len(cad)} intervals; ssb_pipe_kernel duration median {sorted(dur)[len(dur) // 2]:.4f} ms"]
        if prof_line and prof_line.get("ssb_latency_floor"):
            b = prof_line["ssb_latency_floor"]["ssb_ms_coresident"]
            lines.append(f"* the profiled run's own bench line: ssb_ms_coresident {b:.4f} ms, ms_per_step "
                         f"{prof_line['ms_per_step']:.4f} ({100 * (b / med - 1):+.1f} % against the trace)")
bench = None
blog = f"gpurun_out/bench_{TAG}.log"
if os.path.exists(blog):
    for ln in open(blog):
        if ln.startswith("{"):
            bench = json.loads(ln)
    if bench:
        json.dump(bench, open(f"{OUT}/{TAG}_bench.json", "w"), indent=1)
        lines += ["", "## bench.py line", "", "```", json.dumps(bench), "```"]
fetch = counters(f"gpurun_out/pmcf_{TAG}", "FETCH_SIZE")
write = counters(f"gpurun_out/pmcw_{TAG}", "WRITE_SIZE")
pmc = {}
for k in sorted(set(fetch) | set(write)):
    if k not in ENGINE:
        continue
    fk = sorted(fetch.get(k, []))
    wk = sorted(write.get(k, []))
    f_med = fk[len(fk) // 2] * 1024 if fk else None
    w_med = wk[len(wk) // 2] * 1024 if wk else None
    pmc[k] = {"launches": max(len(fk), len(wk)), "fetch_size_bytes_raw": f_med, "write_size_bytes": w_med,
              "fetch_bytes_corrected": 2 * f_med if f_med is not None else None,
              "traffic_bytes": (2 * f_med + w_med) if (f_med is not None and w_med is not None) else None}
if pmc:
    json.dump({"tag": TAG, "command": "bench.py --steps 5 --warmup 1 --no-cpu-baseline (all stages)",
               "correction": "FETCH_SIZE x2 (gfx950 wide coalesced reads), KiB -> bytes", "kernels": pmc},
              open(f"{OUT}/{TAG}_hbm_pmc.json", "w"), indent=1)
    lines += ["", "## HBM traffic per launch (median; FETCH_SIZE doubled per MI355X_MICROARCH.md)", "",
              "| kernel | FETCH raw MB | fetch corrected MB | WRITE MB | traffic MB |", "|---|---|---|---|---|"]
    for k, v in pmc.items():
        def mb(x):
            return f"{x / 1e6:.1f}" if x is not None else "-"
        lines.append(f"| {k} | {mb(v['fetch_size_bytes_raw'])} | {mb(v['fetch_bytes_corrected'])} | "
                     f"{mb(v['write_size_bytes'])} | {mb(v['traffic_bytes'])} |")
open(f"{OUT}/{TAG}_summary.md", "w").write("\n".join(lines) + "\n")
print("\n".join(lines))
