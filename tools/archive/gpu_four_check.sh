#!/bin/bash
# Product check of the persistent four-step selection: 32768 / 65536 parity tests, then configs[4] lines at 5 and 200 kHz
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stats_exact.py tests/test_gpu_any_n.py tests/test_gpu_stats_geometry.py -m gpu -x -q --timeout 120 --timeout-method thread -k "65536 or 32768 or golden or async or pipelined" > gpurun_out/fc_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/fc_tests.log; exit 1; }
tail -n 1 gpurun_out/fc_tests.log
for f in 5 200 5 200; do timeout -k 10 200 python bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-labelled --config c5 --focus $f > gpurun_out/fc_$f.json 2> gpurun_out/fc_$f.err || { echo "bench failed"; tail -5 gpurun_out/fc_$f.err; exit 1; }
echo "focus $f: $(tail -n 1 gpurun_out/fc_$f.json | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["kernel_ms"])')"; done
