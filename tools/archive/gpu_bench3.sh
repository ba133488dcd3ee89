#!/bin/bash
# three default bench lines (c3 headline), no CPU baseline
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-labelled > gpurun_out/b3.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/b3.log; exit 1; }
  tail -1 gpurun_out/b3.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); k=d['kernel_ms']; print(d['value'], d['ms_per_step'], k, d['roofline_isolated']['frac'], d['ssb_latency_floor']['ssb_ms_alone'])"
done
