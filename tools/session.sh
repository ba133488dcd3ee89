#!/bin/bash
# r5ay: narrow statistics phase stamps at HEAD (diagnostic build -DSDRG_STATS_STAMPS=1): c2 (4096 x 16384 CS8, 5 kHz)
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
L=$PWD/sdr-for-android-lib_amd/lib/libsdrg_stamps.so
SDRG_LIB_PATH=$L timeout -k 10 120 python tools/kernel_lab.py --stages spectrum+stats --calls 3 > gpurun_out/r5ay_sstamp.log 2>&1 || { echo failed; tail gpurun_out/r5ay_sstamp.log; exit 1; }
cat gpurun_out/r5ay_sstamp.log
