#!/bin/bash
# SSB per-role cycles (stamps): product library vs the serial roles on all 64 lanes (fe7) / the LPF only (fe2)
export TMPDIR=/tmp
run() { SDRG_LIB_PATH=$3 SDRG_PIPE_STAMPS=1 SDRG_PIPE_SKIP=$1 timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --stages ssb > gpurun_out/ssbdiag.log 2>&1 || exit 1; echo "== skip $1 $2"; grep stamps gpurun_out/ssbdiag.log | tail -12 | head -3 | cut -c1-90; }
run 0 "product" "" || exit 1
run 0 "fe7" sdr-for-android-lib_amd/lib/libsdrg_fe7.so || exit 1
run 0 "fe2" sdr-for-android-lib_amd/lib/libsdrg_fe2.so || exit 1
run 0xFFD "LPF only, fe2" sdr-for-android-lib_amd/lib/libsdrg_fe2.so || exit 1
run 0xFFD "LPF only, product" "" || exit 1
