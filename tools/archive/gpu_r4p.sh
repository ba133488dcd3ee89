#!/bin/bash
# round 4: where the driver's 20-step line loses to the steady step: kernel trace of `bench.py --warmup 5 --steps 20`
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tr20 -o run --output-format csv -- python3 bench.py --warmup 5 --steps 20 --no-labelled --no-cpu-baseline > gpurun_out/tr20.json 2>gpurun_out/tr20.err || { tail -5 gpurun_out/tr20.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/tr20.json')); print('line', d['value'], d['ms_per_step'])"
python3 tools/lab/trace_region.py gpurun_out/tr20/run_kernel_trace.csv 20
