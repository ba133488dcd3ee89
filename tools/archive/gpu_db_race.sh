#!/bin/bash
# the statistics exactness tests at 65536 points, repeated (fresh engines: staging buffers allocated and zeroed per test)
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2 3 4; do
  timeout -k 10 120 python -u -m pytest tests/test_gpu_stats_exact.py -m gpu -q --timeout 60 --timeout-method thread > gpurun_out/race_$i.log 2>&1; echo "run $i rc=$? $(tail -n 1 gpurun_out/race_$i.log)"
done
