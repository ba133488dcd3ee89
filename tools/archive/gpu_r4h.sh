#!/bin/bash
# round 4: the one-rank RCCL bench path, per-step gathers asynchronous (default) vs synchronous, alternating
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  for m in "--gather-mode async" "--gather-mode sync"; do
    timeout -k 10 200 python bench.py --process-group --steps 100 --warmup 20 --no-cpu-baseline $m > gpurun_out/r4h.json 2> gpurun_out/r4h.err || { tail -20 gpurun_out/r4h.err; exit 1; }
    echo "pg $m $(python3 -c "import json; d=json.load(open('gpurun_out/r4h.json')); print(d['value'], d['ms_per_step'], d['kernel_ms'], d.get('gather_check'), d.get('backend'))")"
  done
done
