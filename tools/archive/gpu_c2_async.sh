#!/bin/bash
# BASELINE configs[1] (c2: FFT + statistics) with asynchronous statistics beside a one-workgroup-per-CU spectrum
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "pipelined or async" > gpurun_out/c2a_tests.log 2>&1 || { echo "tests failed"; tail -20 gpurun_out/c2a_tests.log; exit 1; }
tail -1 gpurun_out/c2a_tests.log
run() {
  timeout -k 10 200 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-labelled --config c2 --stats-async $2 > gpurun_out/c2a_$1.json 2> gpurun_out/c2a_$1.err || { echo "bench $1 failed"; tail -5 gpurun_out/c2a_$1.err; exit 1; }
  echo "$1 $(tail -1 gpurun_out/c2a_$1.json | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["kernel_ms"])')"
}
for r in a b; do run async_$r 1 && run sync_$r 0 || exit 1; done
bash tools/gpu_wave_ab.sh
