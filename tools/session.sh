#!/bin/bash
# r5bg: SSB workgroups' start skew and loop cycles per co-resident stage set (lab stamps build)
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
L=$PWD/sdr-for-android-lib_amd/lib/libsdrg_labt.so
SDRG_LIB_PATH=$L SDRG_PIPE_STAMPS=1 timeout -k 10 300 python3 tools/lab/coresidency_stamps.py > gpurun_out/r5bg.log 2>&1 || { tail gpurun_out/r5bg.log; exit 1; }
awk '/^BLOCK/{b=$2; getline; next} /workgroup loop starts/{if(b) w[b]=$0} /wave 1 LPF/{if(b){print b": "w[b]; print b": "$0; b=""}}' gpurun_out/r5bg.log | sed 's/\[sdrg stamps\]//' | cut -c1-250
