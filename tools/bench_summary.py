"""Print the headline of a bench.py JSON line: value, ms/step, per-kernel ms, roofline fractions, labelled lines."""
import json
import sys

for path in sys.argv[1:]:
    lines = [l for l in open(path) if l.startswith('{"metric"')]
    if not lines:
        print(path, "no bench line")
        continue
    d = json.loads(lines[-1])
    k = d.get("kernel_ms", {})
    print(f"{path}: {d['value'] / 1e3:.1f} G {d['ms_per_step']:.4f} ms/step | spec {k.get('spectrum_ms', 0):.4f} "
          f"stats {k.get('stats_ms', 0):.4f} ssb {k.get('ssb_ms', 0):.4f} | roofline {d['roofline']['frac']} "
          f"iso {d.get('roofline_isolated', {}).get('frac')} d2d {d.get('hbm_measured', {}).get('d2d_copy_GBs')}")
    fl = d.get("ssb_latency_floor")
    if fl:
        print(f"   ssb alone {fl['ssb_ms_alone']} coresident {fl['ssb_ms_coresident']}")
    for name, l in d.get("labelled", {}).items():
        extra = " ".join(f"{x} {l[x]}" for x in ("spectrum_ms", "stats_ms", "ssb_ms", "stats_async") if x in l)
        print(f"   {name}: {l['value'] / 1e3:.1f} G {l['ms_per_step']} ms {extra}")
    if "cpu_baseline" in d:
        print("   cpu", d["cpu_baseline"].get("value"), d["cpu_baseline"].get("cores"))
