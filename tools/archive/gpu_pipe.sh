#!/bin/bash
export TMPDIR=/tmp
for p in 0 1 0 1; do
  timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --pipelined $p > gpurun_out/b.log 2>&1 || { tail -5 gpurun_out/b.log; exit 1; }
  echo "pipelined=$p $(grep metric gpurun_out/b.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['kernel_ms'], d['roofline']['frac'])")"
done
