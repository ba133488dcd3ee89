#!/bin/bash
# r5aq: the first steps after a host synchronisation (the driver command's ~250-300 us fixed cost per timed region):
# per-step kernel durations of blocks right after a sync, after 20 ms idle, FFT+stats-only and SSB-only blocks
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/lab/startup_trace.py > gpurun_out/r5aq_plain.log 2>&1 || { tail gpurun_out/r5aq_plain.log; exit 1; }
cat gpurun_out/r5aq_plain.log
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r5aq_tr -o run --output-format csv -- python3 tools/lab/startup_trace.py > gpurun_out/r5aq_tr.log 2>&1 || { tail gpurun_out/r5aq_tr.log; exit 1; }
grep '^P' gpurun_out/r5aq_tr.log
python3 tools/lab/startup_blocks.py gpurun_out/r5aq_tr/run_kernel_trace.csv 8
