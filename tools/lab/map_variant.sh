#!/bin/bash
# lab: SSB role maps for the NCO + 127-tap variant (bench --ssb-variant nco127), alternating processes
mkdir -p gpurun_out
for rep in 1 2; do
  for m in ${MAPS:-7B984A653210 5B984A673210 8B974A653210}; do
    SDRG_PIPE_MAP=$m timeout -k 10 120 python bench.py --ssb-variant nco127 --no-labelled --no-cpu-baseline --steps 100 --warmup 100 > gpurun_out/mapv_$m.log 2>&1 || { echo "map $m failed"; exit 1; }
    echo "$m $(tail -1 gpurun_out/mapv_$m.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["kernel_ms"])')"
  done
done
