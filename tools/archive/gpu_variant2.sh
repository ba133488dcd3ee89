#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ssb_variant.py -x -q --timeout 120 --timeout-method thread > gpurun_out/variant_tests.log 2>&1; rc=$?
echo "pytest rc $rc" >> gpurun_out/variant_tests.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/variant_tests.log; exit 1; }
tail -2 gpurun_out/variant_tests.log
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --ssb-variant nco127 > gpurun_out/bench_nco.log 2>&1 || { echo bench variant failed; tail -5 gpurun_out/bench_nco.log; exit 1; }
SDRG_PIPE_STAMPS=1 timeout -k 10 200 python bench.py --steps 3 --warmup 1 --ssb-variant nco127 > gpurun_out/bench_nco_stamps.log 2>&1 || { echo stamps failed; exit 1; }
grep "stamps" gpurun_out/bench_nco_stamps.log | tail -12
cat gpurun_out/bench_nco.log | grep metric | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['value'], d['ms_per_step'], d['kernel_ms'], d['roofline']['frac'], d.get('ssb_variant'))"
