"""Lab: join tools/lab/ssb_boundary.py's stamps (per call: first entry, first loop start, last loop end, s_memrealtime
in 10 ns units) with the rocprofv3 kernel trace's ssb_pipe_kernel start / end (ns) of the same run, in call order.

The two clocks are fitted with one offset per run: the smallest (trace start - entry) over all calls, so that every
dispatch-to-entry delay is >= 0 and the smallest is 0 (both clocks tick the same 100 MHz reference if this is sound:
the printed spread shows it).  Per block: trace duration, (entry - trace start) - min, loop span, (trace end - loop end).
python tools/lab/ssb_boundary_join.py LOG TRACE_CSV
"""
import csv
import re
import statistics
import sys


def main():
    log, trace = sys.argv[1], sys.argv[2]
    blocks, cur = {}, None
    for line in open(log):
        if line.startswith("BLOCK"):
            cur = line.split()[1]
            blocks[cur] = []
        elif cur and "abs entry" in line:
            m = re.search(r"abs entry (\d+) loop (\d+) end (\d+)", line)
            blocks[cur].append(tuple(int(x) * 10 for x in m.groups()))
    rows = []
    with open(trace) as fh:
        for r in csv.DictReader(fh):
            if "ssb_pipe_kernel" in r["Kernel_Name"]:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows.sort()
    n = sum(len(v) for v in blocks.values())
    tail = rows[-n:]
    i = 0
    pairs = {}
    for name, calls in blocks.items():
        pairs[name] = list(zip(calls, tail[i:i + len(calls)]))
        i += len(calls)
    offs = [t[0] - s[0] for v in pairs.values() for s, t in v]
    off = min(offs)
    print(f"clock offset {off} ns; (trace start - entry) spread {max(offs) - off} ns over {len(offs)} calls")
    for name, v in pairs.items():
        cols = []
        for s, t in v[len(v) // 3:-1]:  # past the first third of the block (the start after a synchronisation)
            entry, loop, end = (x + off for x in s)
            cols.append(((t[1] - t[0]) / 1e3, (entry - t[0]) / 1e3, (loop - entry) / 1e3, (end - loop) / 1e3,
                         (t[1] - end) / 1e3))
        med = [statistics.median(c[i] for c in cols) for i in range(5)]
        print(f"== {name} ({len(cols)} calls, medians): trace {med[0]:.1f} us | start->entry {med[1]:.1f} | entry->loop "
              f"{med[2]:.1f} | loop span {med[3]:.1f} | loop end->trace end {med[4]:.1f} us")
    # the gap between consecutive SSB kernels in each block (trace end -> next trace start)
    for name, v in pairs.items():
        ts = [t for _, t in v[len(v) // 3:]]
        gaps = [(b[0] - a[1]) / 1e3 for a, b in zip(ts, ts[1:])]
        print(f"== {name}: kernel-to-kernel gap median {statistics.median(gaps):.1f} us")


if __name__ == "__main__":
    main()
