#!/bin/bash
# r5bc: SSB workgroups' loop start skew and span (lab stamps build), c3 step vs the SSB stage alone
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
L=sdr-for-android-lib_amd/lib/libsdrg_labt.so
for st in all ssb; do
  SDRG_LIB_PATH=$L SDRG_PIPE_STAMPS=1 timeout -k 10 200 python bench.py --steps 40 --warmup 3 --no-cpu-baseline --no-labelled --stages $st > gpurun_out/r5bc_$st.log 2>&1 || { echo "stamps $st failed"; tail gpurun_out/r5bc_$st.log; exit 1; }
  echo "== $st"
  grep "sdrg stamps" gpurun_out/r5bc_$st.log | grep -E "workgroup|LPF" | tail -3 | sed 's/.*stamps\]//'
done
