#!/bin/bash
# r6w2: narrow statistics phase stamps at 1024 and 4096 frames (16384 / 5 kHz): the uncontended frame against the
# product's four waves per SIMD
set -o pipefail
export TMPDIR=/tmp
for b in 1024 4096; do
  SDRG_LIB_PATH=sdr-for-android-lib_amd/lib/libsdrg_stamps.so timeout -k 10 120 python tools/lab/stats_time.py 16384 5 $b 5 2>&1 | tail -2 || exit 1
done
