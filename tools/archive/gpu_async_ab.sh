#!/bin/bash
# SDRG_PIPELINE_STATS_ASYNC: GPU parity (every pipelined mode bit-identical to the joined schedule), then the bench
# lines with and without it, alternating.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_engine_api.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/aab_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/aab_tests.log; exit 1; }
tail -1 gpurun_out/aab_tests.log
run() {  # tag async extra
  timeout -k 10 200 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-labelled --stats-async $2 $3 > gpurun_out/aab_$1.json 2> gpurun_out/aab_$1.err || { echo "bench $1 failed"; tail -5 gpurun_out/aab_$1.err; exit 1; }
  echo "$1 $(tail -1 gpurun_out/aab_$1.json | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["kernel_ms"])')"
}
for r in a b; do
  run c3_async_$r 1 "" && run c3_sync_$r 0 "" || exit 1
  run c2_async_$r 1 "--config c2" && run c2_sync_$r 0 "--config c2" || exit 1
  run c5_200_async_$r 1 "--config c5 --focus 200" && run c5_200_sync_$r 0 "--config c5 --focus 200" || exit 1
  run c5_5_async_$r 1 "--config c5 --focus 5" && run c5_5_sync_$r 0 "--config c5 --focus 5" || exit 1
done
