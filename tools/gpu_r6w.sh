#!/bin/bash
# r6w: narrow statistics alone at 16384 / 5 kHz for 1024 / 2048 / 4096 / 8192 frames (is the kernel bound by a frame's
# latency or by the SIMDs' issue?)
set -o pipefail
export TMPDIR=/tmp
for b in 1024 2048 4096 8192; do
  timeout -k 10 120 python tools/lab/stats_time.py 16384 5 $b 50 2>&1 | tail -1 || exit 1
done
