#!/bin/bash
# persistent spectrum grid (SDRG_SPECTRUM_GRID) under SSB co-residency: default 2 x CUs vs 1 x CUs and others
export TMPDIR=/tmp
mkdir -p gpurun_out
for g in 0 256 384 0 256 768; do
  if [ $g = 0 ]; then E=""; else E="SDRG_SPECTRUM_GRID=$g"; fi
  env $E timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/grid_$g.log 2>&1 || { echo "grid $g failed"; tail -5 gpurun_out/grid_$g.log; exit 1; }
  echo "grid $g $(tail -1 gpurun_out/grid_$g.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["kernel_ms"], d["roofline"]["frac"], d["roofline_isolated"]["frac"])')"
done
