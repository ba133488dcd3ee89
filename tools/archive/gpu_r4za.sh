#!/bin/bash
# round 4: the persistent four-step kernels beside the multi-frame wide statistics (pw1) against the one-tile-per-
# workgroup kernels there (pw0, the round-3 choice, measured beside the single-frame wide kernel): configs[4] 200 kHz
# (pw1 was built from a temporary patch: launch_spectrum passing persistent = true beside the wide statistics; not kept)
export TMPDIR=/tmp
mkdir -p gpurun_out
D=sdr-for-android-lib_amd/lib
for i in 1 2 3; do
  for v in pw0 pw1; do
    SDRG_LIB_PATH=$D/libsdrg_$v.so timeout -k 10 200 python bench.py --config c5 --focus 200 --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/r4za.json 2>/dev/null || exit 1
    echo "$v 200 kHz $(python3 -c "import json; d=json.load(open('gpurun_out/r4za.json')); print(d['value'], d['ms_per_step'], d['kernel_ms'])")"
  done
done
