#!/bin/bash
# per-role SSB cycles (stamps) of the product and the low-pass lab variants (libsdrg_lpfN.so), all roles running
# and the low-pass wave alone (others skipped)
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in product "$@"; do
  lib=""; [ "$n" = product ] || lib=sdr-for-android-lib_amd/lib/libsdrg_$n.so
  for skip in 0 0xFFD; do
    SDRG_LIB_PATH=$lib SDRG_PIPE_STAMPS=1 SDRG_PIPE_SKIP=$skip timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --stages ssb > gpurun_out/lpfv.log 2>&1 || exit 1
    echo "$n skip=$skip $(grep stamps gpurun_out/lpfv.log | tail -12 | awk '{printf "%s:%d ", $5, $8/1000} END {print "loop:" $11/1000}')"
  done
done
