#!/bin/bash
# round 4: issue priority 1 for the spectrum waves (kp1) against none (kp0), with the statistics after the spectrum
# (async 0) or beside the next call's spectrum (async 1): configs[1] line (FFT + statistics, no SSB), alternating
export TMPDIR=/tmp
mkdir -p gpurun_out
D=sdr-for-android-lib_amd/lib
for i in 1 2; do
  for v in kp0 kp1; do
    for a in 0 1; do
      SDRG_LIB_PATH=$D/libsdrg_$v.so timeout -k 10 200 python bench.py --stages spectrum+stats --steps 300 --warmup 20 --stats-async $a --no-labelled --no-cpu-baseline > gpurun_out/r4q.json 2>/dev/null || exit 1
      echo "$v async=$a $(python3 -c "import json; d=json.load(open('gpurun_out/r4q.json')); print(d['value'], d['ms_per_step'], d['kernel_ms'])")"
    done
  done
done
