#!/bin/bash
# the labelled bench lines: BASELINE configs[1] (c2), configs[2] (the NCO variant), configs[4] (c5 at 5 and 200 kHz)
export TMPDIR=/tmp
mkdir -p gpurun_out
b() { timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/cfg.log 2>&1 || { echo "failed: $*"; tail -5 gpurun_out/cfg.log; exit 1; }
      grep metric gpurun_out/cfg.log >> gpurun_out/configs.jsonl; grep metric gpurun_out/cfg.log | python3 -c "
import sys, json; d = json.loads(sys.stdin.read()); print('$*', d['value'], d['ms_per_step'], d['kernel_ms'], d['roofline']['frac'], d['roofline_isolated']['frac'], d['hbm_measured'])"; }
rm -f gpurun_out/configs.jsonl
b
b --config c2
b --ssb-variant nco127
b --config c5
b --config c5 --focus 200
