#!/bin/bash
# r5ac: the driver's command (--steps 20 --warmup 5) against the pre-roll length (bench.py --prewarm-ms)
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for p in 100 300 1000; do
    o=gpurun_out/r5ac_p${p}_$i
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --prewarm-ms $p --no-labelled --no-cpu-baseline > $o.json 2> $o.err || { tail $o.err; exit 1; }
    echo "prewarm $p: $(python tools/bench_summary.py $o.json | head -2 | cut -d: -f2- | tr '\n' ' ')"
  done
done
