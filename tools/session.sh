#!/bin/bash
# r5bk: statistics that co-reside with the spectrum and SSB workgroups (lab build "co": SSB taps in 2 copies (-3 KB LDS),
# narrow statistics with its StatsState in LDS, 2 loads in flight, 48 VGPRs): statistics + SSB tests on it, the SSB
# start skew (stamps), then the c3 line against the product, alternating
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
L=$PWD/sdr-for-android-lib_amd/lib/libsdrg_co.so
LAB_ALL_ONLY=1 SDRG_LIB_PATH=$L SDRG_PIPE_STAMPS=1 timeout -k 10 200 python3 tools/lab/coresidency_stamps.py > gpurun_out/r5bk_co.log 2>&1 || { tail gpurun_out/r5bk_co.log; exit 1; }
awk '/^BLOCK/{b=$2; getline; next} /workgroup loop starts/{if(b) w[b]=$0} /wave 1 LPF/{if(b){print w[b]; print $0; b=""}}' gpurun_out/r5bk_co.log | sed 's/\[sdrg stamps\]//; s/work [0-9]* loop/loop/g' | cut -c1-220
bash tools/ab.sh -r 3 -o r5bk -t "tests/test_gpu_parity.py tests/test_gpu_stats_exact.py tests/test_gpu_stats_geometry.py tests/test_gpu_ssb_schedule.py" base co -- \
  python bench.py --no-cpu-baseline --no-labelled
