#!/bin/bash
# statistics parity (every test that checks records) and the labelled c2 / c5 lines
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_any_n.py tests/test_gpu_edges.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/stats_parity.log 2>&1 || { echo "parity failed"; tail -30 gpurun_out/stats_parity.log; exit 1; }
tail -1 gpurun_out/stats_parity.log
for a in ${BENCHES:-"--config c5 --focus 200" "--config c5 --focus 5" "--config c2"}; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline $a > gpurun_out/stats_bench.log 2>&1 || { echo "bench $a failed"; tail -5 gpurun_out/stats_bench.log; exit 1; }
  echo "$a: $(tail -1 gpurun_out/stats_bench.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["kernel_ms"])')"
done
