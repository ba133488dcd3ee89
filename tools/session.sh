#!/bin/bash
# r5f: the 64-lane serial roles' own rate in the ssb64 front (loader skipped, wrong results): per-role stamps
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
T=r5f
D=sdr-for-android-lib_amd/lib
SDRG_SSB64_STAMPS=1 SDRG_LIB_PATH=$D/libsdrg_ssb64skip.so timeout -k 10 200 python bench.py --stages ssb --steps 40 --warmup 5 --no-cpu-baseline --no-labelled --prewarm-ms 0 > gpurun_out/${T}_st.json 2> gpurun_out/${T}_st.err || { tail -5 gpurun_out/${T}_st.err; exit 1; }
grep "ssb64 stamps" gpurun_out/${T}_st.err | tail -1
SDRG_PIPE_STAMPS=1 SDRG_LIB_PATH=$D/libsdrg_ssb64skip.so SDRG_SSB64=0 timeout -k 10 200 python bench.py --stages ssb --steps 40 --warmup 5 --no-cpu-baseline --no-labelled --prewarm-ms 0 > gpurun_out/${T}_st16.json 2> gpurun_out/${T}_st16.err || { tail -5 gpurun_out/${T}_st16.err; exit 1; }
grep "sdrg stamps" gpurun_out/${T}_st16.err | tail -12
