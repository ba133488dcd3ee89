#!/bin/bash
# GPU test suite + per-role SSB cycles (stamps) + a short default bench
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/gpu_tests.log | head -20; exit 1; }
SDRG_PIPE_STAMPS=1 timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --stages ssb > gpurun_out/ssbdiag.log 2>&1 || exit 1
grep stamps gpurun_out/ssbdiag.log | tail -12 | cut -c1-90
SDRG_PIPE_STAMPS=1 SDRG_PIPE_SKIP=0xFFD timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --stages ssb > gpurun_out/ssbdiag2.log 2>&1 || exit 1
grep stamps gpurun_out/ssbdiag2.log | tail -12 | sed -n 2p | cut -c1-90
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_quick.log 2>&1 || exit 1
tail -1 gpurun_out/bench_quick.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'ms', d['ms_per_step'], 'kernel_ms', d['kernel_ms'], 'ssb floor', d.get('ssb_latency_floor',{}).get('ssb_ms_alone'))"
