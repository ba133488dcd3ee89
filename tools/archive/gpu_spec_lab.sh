#!/bin/bash
# spectrum16k: parity (every test that checks N = 16384 spectra) and its isolated / c2 timings
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/spec_parity.log 2>&1 || { echo "parity failed"; tail -30 gpurun_out/spec_parity.log; exit 1; }
tail -1 gpurun_out/spec_parity.log
for f in CS8 CS16; do
  timeout -k 10 120 python tools/kernel_lab.py --stages spectrum --calls 30 --fmt $f > gpurun_out/spec_lab.log 2>&1 || { echo "lab failed"; tail -5 gpurun_out/spec_lab.log; exit 1; }
  echo "$f $(tail -1 gpurun_out/spec_lab.log)"
done
timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --config c2 > gpurun_out/spec_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/spec_bench.log; exit 1; }
tail -1 gpurun_out/spec_bench.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("c2", d["value"], d["ms_per_step"], d["kernel_ms"], d.get("roofline_isolated",{}).get("frac"))'
