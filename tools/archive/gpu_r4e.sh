#!/bin/bash
# round 4: phase stamps of the multi-frame wide statistics kernel across lab variants (SDRG_MW_STAMPS=1)
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in ${@:-mwst}; do
  echo "== $v"
  SDRG_LIB_PATH=sdr-for-android-lib_amd/lib/libsdrg_$v.so timeout -k 10 60 python tools/lab/stats_time.py 65536 200 1024 3 2>&1 | tail -2
done
