"""Lab: the timed region of a short bench run in a rocprofv3 kernel trace (tools/gpu_r4p.sh).

The timed steps follow the last host synchronisation before the isolated-spectrum phase: the GPU idles there (the
bench synchronises, resets its timing statistics and barriers), so the region starts at the first dispatch after the
last idle gap longer than --gap-us that precedes the K-th-from-last ssb_pipe_kernel of the STAGE_ALL steps.  Prints
each stream's kernels of the first and last steps with their start/end relative to the region's first dispatch, the
SSB kernels' start-to-start intervals, and the region's span against K x the steady interval.
python tools/lab/trace_region.py TRACE_CSV K
"""
import csv
import sys


def short(name):
    for k in ("ssb_pipe_kernel", "spectrum16k_kernel", "stats_narrow_kernel", "stats_wide", "spectral_pulse_kernel",
              "audio_pulse_kernel", "pulse_reset_kernel", "four_step"):
        if k in name:
            return k
    return name[:40]


def main():
    path, K = sys.argv[1], int(sys.argv[2])
    rows = []
    with open(path) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                         r.get("Queue_Id", "")))
    rows.sort()
    ssb = [i for i, r in enumerate(rows) if "ssb_pipe_kernel" in r[2]]
    # last run of >= 5 consecutive spectrum launches with no SSB between = the isolated phase
    runs = []
    i = 0
    while i < len(rows):
        if "spectrum16k" in rows[i][2]:
            j = i
            while j < len(rows) and ("spectrum16k" in rows[j][2]):
                j += 1
            if j - i >= 5:
                runs.append(i)
            i = j
        else:
            i += 1
    iso = runs[-1] if runs else len(rows)
    timed_ssb = [k for k in ssb if k < iso][-K:]
    # region start: the first dispatch after the last idle gap (> 50 us) before the first timed SSB kernel
    region_start = None
    for idx in range(timed_ssb[0], -1, -1):
        if idx == 0:
            region_start = 0
            break
        gap = rows[idx][0] - max(r[1] for r in rows[max(0, idx - 40):idx])
        if gap > 50_000:
            region_start = idx
            break
    t0 = rows[region_start][0]
    # the region ends at the last kernel before the isolated phase
    ends = [r[1] for r in rows[region_start:iso]]
    t1 = max(ends)
    print(f"region: dispatch {region_start}..{iso - 1}, span {(t1 - t0) / 1e3:.1f} us for {K} steps "
          f"({(t1 - t0) / 1e3 / K:.2f} us per step)")
    starts = [rows[k][0] for k in timed_ssb]
    iv = [(b - a) / 1e3 for a, b in zip(starts, starts[1:])]
    iv_sorted = sorted(iv)
    print(f"SSB start-to-start: median {iv_sorted[len(iv) // 2]:.1f} us, first {iv[0]:.1f}, last {iv[-1]:.1f}; "
          f"SSB kernel durations first {(rows[timed_ssb[0]][1] - rows[timed_ssb[0]][0]) / 1e3:.1f}, "
          f"last {(rows[timed_ssb[-1]][1] - rows[timed_ssb[-1]][0]) / 1e3:.1f} us")
    print(f"first SSB starts {(starts[0] - t0) / 1e3:.1f} us into the region; last SSB ends "
          f"{(t1 - rows[timed_ssb[-1]][1]) / 1e3:.1f} us before the region's end")
    print("first dispatches:")
    for r in rows[region_start:region_start + 12]:
        print(f"  {(r[0] - t0) / 1e3:9.1f} {(r[1] - t0) / 1e3:9.1f}  q{r[3]}  {short(r[2])}")
    print("last dispatches:")
    for r in rows[iso - 12:iso]:
        print(f"  {(r[0] - t0) / 1e3:9.1f} {(r[1] - t0) / 1e3:9.1f}  q{r[3]}  {short(r[2])}")


if __name__ == "__main__":
    main()
