#!/bin/bash
# round 4: the four-step FFT waves at issue priority 1 (fs1) over the asynchronous statistics beside them, against 0 (fs0):
# the configs[4] lines at 5 and 200 kHz, alternating
export TMPDIR=/tmp
mkdir -p gpurun_out
D=sdr-for-android-lib_amd/lib
for i in 1 2 3; do
  for v in fs0 fs1; do
    for f in 5 200; do
      SDRG_LIB_PATH=$D/libsdrg_$v.so timeout -k 10 200 python bench.py --config c5 --focus $f --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/r4y.json 2>/dev/null || exit 1
      echo "$v $f kHz $(python3 -c "import json; d=json.load(open('gpurun_out/r4y.json')); print(d['value'], d['ms_per_step'], d['kernel_ms'])")"
    done
  done
done
