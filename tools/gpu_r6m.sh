#!/bin/bash
# r6m: (1) the driver's 20-step command, HEAD's SSB + spectrum sources (lab build "lab") against round 5's (lab build
# "r5both": csrc/ssb.hip and csrc/spectrum.hip of commit 1eb6060, the rest HEAD), alternating; (2) the wide statistics'
# dB scratch (lab "dbpool", SDRG_MW_DBPOOL=1): statistics GPU tests, the kernel alone at 65536 / 200 kHz, the configs[4]
# 200 kHz line, alternating against "lab".
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=sdr-for-android-lib_amd/lib
tools/ab.sh -r 3 -o r6m lab r5both -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-labelled || exit 1
SDRG_LIB_PATH=$L/libsdrg_dbpool.so timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_stats_exact.py tests/test_gpu_stats_geometry.py tests/test_gpu_parity.py tests/test_gpu_any_n.py \
  > gpurun_out/r6m_tests_dbpool.log 2>&1 || { echo "dbpool tests FAILED"; tail -40 gpurun_out/r6m_tests_dbpool.log; exit 1; }
echo "dbpool: $(tail -1 gpurun_out/r6m_tests_dbpool.log)"
for v in lab dbpool lab dbpool; do
  SDRG_LIB_PATH=$L/libsdrg_$v.so timeout -k 10 120 python tools/lab/stats_time.py 65536 200 1024 30 || exit 1
done
tools/ab.sh -r 2 -o r6m5 lab dbpool -- python bench.py --config c5 --focus 200 --steps 100 --warmup 30 --no-cpu-baseline
