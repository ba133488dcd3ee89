#!/bin/bash
# a short SSB-only run under a tight limit first (a new pipeline schedule), then tools/gpu_quick.sh
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 90 python bench.py --steps 3 --warmup 1 --stages ssb --no-cpu-baseline > gpurun_out/ssb_first.log 2>&1 || { echo "ssb-only run failed rc=$?"; tail -5 gpurun_out/ssb_first.log; exit 1; }
echo "ssb-only run ok"
bash tools/gpu_quick.sh
