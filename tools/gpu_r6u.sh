#!/bin/bash
# r6u: the narrow statistics' staging copy as buffer loads straight into LDS (product build, SDRG_NARROW_DMA=1) against
# the register copy (lab build nodma): statistics GPU tests (bit-exact), the kernel alone, the bench A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=sdr-for-android-lib_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_stats_exact.py tests/test_gpu_stats_geometry.py tests/test_gpu_parity.py tests/test_gpu_edges.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6u_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r6u_tests.log; exit 1; }
tail -1 gpurun_out/r6u_tests.log
for r in 1 2; do
  for v in nodma base; do
    lib=$L/libsdrg.so; [ $v != base ] && lib=$L/libsdrg_$v.so
    for cfg in "16384 5 4096" "65536 5 1024"; do
      SDRG_LIB_PATH=$lib timeout -k 10 120 python tools/lab/stats_time.py $cfg 50 > gpurun_out/r6u_st.log 2>&1 || { echo "stats_time $v failed"; tail gpurun_out/r6u_st.log; exit 1; }
      echo "$v: $(tail -1 gpurun_out/r6u_st.log)"
    done
  done
done
bash tools/ab.sh -r 2 -o r6u nodma base -- python bench.py --steps 200 --warmup 100 --no-cpu-baseline
