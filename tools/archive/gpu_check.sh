#!/bin/bash
# GPU validation: gpu tests (per-test timeout), fftlab (k16), one bench line for the full per-frame work and
# one for the hot path alone (ablation)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "pytest rc $rc" >> gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 5 120 ./tools/fftlab/fftlab 4096 k16 > gpurun_out/fftlab.log 2>&1 || { echo fftlab failed; exit 1; }
cat gpurun_out/fftlab.log
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench.log 2>&1 || { echo bench failed; tail -5 gpurun_out/bench.log; exit 1; }
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --stages hot --no-cpu-baseline > gpurun_out/bench_hot.log 2>&1 || { echo bench hot failed; tail -5 gpurun_out/bench_hot.log; exit 1; }
cat gpurun_out/bench.log gpurun_out/bench_hot.log | grep metric | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['value'], d['ms_per_step'], d['kernel_ms'], d['roofline']['frac'], d.get('cpu_baseline', {}).get('value'))"
