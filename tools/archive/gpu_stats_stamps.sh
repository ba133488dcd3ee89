#!/bin/bash
# diagnostic statistics stamps (libsdrg_stamps.so): c5 / 200 kHz (wide kernel) and c2 (narrow kernel)
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/sdr-for-android-lib_amd/lib/libsdrg_stamps.so
SDRG_LIB_PATH=$L timeout -k 10 120 python tools/kernel_lab.py --stages spectrum+stats --n 65536 --fmt CS16 --streams 1024 --focus 200 --calls 3 > gpurun_out/sstamp.log 2>&1 || { echo failed; tail gpurun_out/sstamp.log; exit 1; }
cat gpurun_out/sstamp.log
SDRG_LIB_PATH=$L timeout -k 10 120 python tools/kernel_lab.py --stages spectrum+stats --calls 3 > gpurun_out/sstamp2.log 2>&1 || { echo failed; tail gpurun_out/sstamp2.log; exit 1; }
cat gpurun_out/sstamp2.log
SDRG_LIB_PATH=$L timeout -k 10 120 python tools/kernel_lab.py --stages spectrum+stats --n 65536 --fmt CS16 --streams 1024 --focus 5 --calls 3 > gpurun_out/sstamp3.log 2>&1 || { echo failed; tail gpurun_out/sstamp3.log; exit 1; }
cat gpurun_out/sstamp3.log
