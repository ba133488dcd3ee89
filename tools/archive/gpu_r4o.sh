#!/bin/bash
# round 4: the product after the narrow statistics' 64-VGPR budget and asynchronous statistics in the c3 line:
# GPU suite, smoke, the driver's command and the default line
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4o_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r4o_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r4o_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4o_smoke.log 2>&1 || { tail -20 gpurun_out/r4o_smoke.log; exit 1; }
tail -1 gpurun_out/r4o_smoke.log
timeout -k 10 300 python bench.py --warmup 5 --steps 20 > gpurun_out/r4o_driverlike.json 2>gpurun_out/r4o_driverlike.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r4o_driverlike.json')); print('driverlike', d['value'], d['ms_per_step'])"
timeout -k 10 300 python bench.py > gpurun_out/r4o_bench.json 2>gpurun_out/r4o_bench.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r4o_bench.json')); l=d['labelled']; print('default', d['value'], d['ms_per_step'], d['kernel_ms'], {k: v['value'] for k, v in l.items()})"
