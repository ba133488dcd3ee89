#!/bin/bash
# GPU check of the NCO/127-tap SSB variant: its parity tests, then the default bench line and the variant's
# separately labelled line (no CPU baseline in either, to keep the call short)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ssb_variant.py tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread > gpurun_out/variant_tests.log 2>&1; rc=$?
echo "pytest rc $rc" >> gpurun_out/variant_tests.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/variant_tests.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/variant_tests.log | tail -30
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/bench_ref.log 2>&1 || { echo bench failed; tail -5 gpurun_out/bench_ref.log; exit 1; }
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --ssb-variant nco127 > gpurun_out/bench_nco.log 2>&1 || { echo bench variant failed; tail -5 gpurun_out/bench_nco.log; exit 1; }
cat gpurun_out/bench_ref.log gpurun_out/bench_nco.log | grep metric | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['value'], d['ms_per_step'], d['kernel_ms'], d['roofline']['frac'], d.get('ssb_variant'))"
