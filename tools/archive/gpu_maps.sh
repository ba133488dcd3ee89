#!/bin/bash
# role-to-wave maps (SDRG_PIPE_MAP, nibble w = role of hardware wave w, SIMD = w % 4): per-role cycles and the
# default bench line for each, alternating
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
for M in "$@"; do
  SDRG_PIPE_MAP=$M SDRG_PIPE_STAMPS=1 timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --stages ssb > gpurun_out/map.log 2>&1 || exit 1
  R=$(grep stamps gpurun_out/map.log | tail -12 | awk '{printf "%s:%d ", $5, $8/1000}')
  SDRG_PIPE_MAP=$M timeout -k 10 300 python bench.py --no-cpu-baseline --no-labelled > gpurun_out/map_bench.log 2>&1 || exit 1
  B=$(tail -1 gpurun_out/map_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['ssb_latency_floor']['ssb_ms_alone'])")
  echo "map $M | $B | $R"
done
done
