#!/bin/bash
# r6i: which roles slow the full-EXEC low-pass loop in the pipeline (lab "copies" alone: 590k cycles per frame with every
# other role skipped, 655k with all of them running): the SSB stage with every role but the low-pass and ONE other
# skipped (SDRG_PIPE_SKIP, wrong results, timing only), and with the serial or the helper roles only.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=sdr-for-android-lib_amd/lib
# 0xFFD & ~X: X = DC 0x1, AGC 0x4, loader 0x8, FIR 0x90, clamp 0x20, EQ 0x40, DES 0xF00; 0xFF8: DC + AGC only;
# 0x5: every helper, no DC / AGC
for m in 0xFFD 0xFFC 0xFF9 0xFF5 0xF6D 0xFDD 0xFBD 0x0FD 0xFF8 0x5 0; do
  SDRG_LIB_PATH=$L/libsdrg_copies.so SDRG_PIPE_STAMPS=1 SDRG_PIPE_SKIP=$m timeout -k 10 200 python tools/lab/step_once.py c_$m 4 > gpurun_out/r6i_$m.log 2>&1 || { echo "stamps $m failed"; tail gpurun_out/r6i_$m.log; exit 1; }
  echo "skip $m: $(grep 'wave 1 LPF' gpurun_out/r6i_$m.log | tail -1 | sed 's/.*steady/steady/')"
done
