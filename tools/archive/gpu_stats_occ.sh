#!/bin/bash
# diagnostic: wide statistics stamps at 4 / 2 / 1 frames per CU (dynamic LDS padded)
export TMPDIR=/tmp
mkdir -p gpurun_out
for kb in 36 72 150; do
  SDRG_STATS_LDS_KB=$kb SDRG_LIB_PATH=$PWD/sdr-for-android-lib_amd/lib/libsdrg_sstamp.so timeout -k 10 120 python tools/kernel_lab.py --stages spectrum+stats --n 65536 --fmt CS16 --streams 1024 --focus 200 --calls 2 > gpurun_out/socc.log 2>&1 || { echo failed; tail gpurun_out/socc.log; exit 1; }
  echo "lds $kb KB"; grep -E "stamps|stats_ms" gpurun_out/socc.log | tail -2
done
