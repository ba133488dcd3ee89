"""Lab: per-step kernel durations of the blocks tools/lab/startup_trace.py runs, from its rocprofv3 kernel trace.

Blocks are separated by idle gaps (no kernel running) longer than 40 us.  For each block after the pre-roll: the
spectrum and SSB kernels' durations in order (us), with the start of each step relative to the block's first
dispatch, marking durations more than 12 % over the block's median.
python tools/lab/startup_blocks.py TRACE_CSV [PREROLL_BLOCKS]
"""
import csv
import statistics
import sys


def main():
    path = sys.argv[1]
    skip = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    rows = []
    with open(path) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    blocks, cur, end = [], [], None
    for r in rows:
        if cur and r[0] - end > 40_000:
            blocks.append(cur)
            cur = []
        end = r[1] if not cur else max(end, r[1])
        cur.append(r)
    if cur:
        blocks.append(cur)
    # keep blocks that run the hot kernels (drops engine set-up and input synthesis)
    blocks = [b for b in blocks if sum(("spectrum16k" in r[2]) or ("ssb_pipe" in r[2]) for r in b) >= 10]
    for bi, b in enumerate(blocks[skip:]):
        t0 = b[0][0]
        span = (max(r[1] for r in b) - t0) / 1e3
        for key in ("spectrum16k", "ssb_pipe"):
            ks = [r for r in b if key in r[2]]
            if not ks:
                continue
            d = [(r[1] - r[0]) / 1e3 for r in ks]
            med = statistics.median(d)
            marks = " ".join(f"{x:.0f}{'*' if x > 1.12 * med else ''}@{(r[0] - t0) / 1e3:.0f}" for x, r in zip(d, ks))
            print(f"block {bi:2d} span {span:7.1f} us {key:11s} median {med:.1f}: {marks}")


if __name__ == "__main__":
    main()
