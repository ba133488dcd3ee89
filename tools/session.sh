#!/bin/bash
# r5bh: SSB workgroup start skew with the c3 step's statistics asynchronous (mode 6) or on the main stream (mode 2)
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
L=$PWD/sdr-for-android-lib_amd/lib/libsdrg_labt.so
for m in 6 2 6 2; do
  LAB_ALL_ONLY=1 LAB_PIPE_MODE=$m SDRG_LIB_PATH=$L SDRG_PIPE_STAMPS=1 timeout -k 10 200 python3 tools/lab/coresidency_stamps.py > gpurun_out/r5bh_$m.log 2>&1 || { tail gpurun_out/r5bh_$m.log; exit 1; }
  echo "mode $m:"
  awk '/^BLOCK/{b=$2; getline; next} /workgroup loop starts/{if(b) w[b]=$0} /wave 1 LPF/{if(b){print w[b]; print $0; b=""}}' gpurun_out/r5bh_$m.log | sed 's/\[sdrg stamps\]//; s/work [0-9]* loop/loop/g' | cut -c1-220
done
