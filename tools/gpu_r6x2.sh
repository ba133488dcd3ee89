#!/bin/bash
# r6x2: the narrow pool's logs side by side (product, SDRG_NARROW_POOL_ILP=1) against one per branch (lab build noilp):
# statistics GPU tests (bit-exact), then the kernel alone, alternating
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=sdr-for-android-lib_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_stats_exact.py tests/test_gpu_stats_geometry.py tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_any_n.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6x2_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r6x2_tests.log; exit 1; }
tail -1 gpurun_out/r6x2_tests.log
for r in 1 2 3; do
  for v in noilp base; do
    lib=$L/libsdrg.so; [ $v != base ] && lib=$L/libsdrg_$v.so
    for cfg in "16384 5 4096" "16384 5 1024" "65536 5 1024"; do
      SDRG_LIB_PATH=$lib timeout -k 10 120 python tools/lab/stats_time.py $cfg 50 > gpurun_out/r6x2_st.log 2>&1 || { echo "stats_time $v failed"; tail gpurun_out/r6x2_st.log; exit 1; }
      echo "$v: $(tail -1 gpurun_out/r6x2_st.log | cut -c1-60)"
    done
  done
done
