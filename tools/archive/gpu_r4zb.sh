#!/bin/bash
# round 4: the asynchronous wide statistics on a CU subset (lab SDRG_STATS_CUS: e even CU-mask bits, h low half, t three
# of every four), the four-step FFT unmasked, against no mask (-): configs[4] 200 kHz
# (libsdrg_pw0 was built from a temporary patch: s_stats created by hipExtStreamCreateWithCUMask per SDRG_STATS_CUS; not kept)
export TMPDIR=/tmp
mkdir -p gpurun_out
D=sdr-for-android-lib_amd/lib
for i in 1 2; do
  for v in - e h t; do
    if [ "$v" = "-" ]; then unset SDRG_STATS_CUS; else export SDRG_STATS_CUS=$v; fi
    SDRG_LIB_PATH=$D/libsdrg_pw0.so timeout -k 10 200 python bench.py --config c5 --focus 200 --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/r4zb.json 2>/dev/null || exit 1
    echo "cus=$v 200 kHz $(python3 -c "import json; d=json.load(open('gpurun_out/r4zb.json')); print(d['value'], d['ms_per_step'], d['kernel_ms'])")"
  done
done
