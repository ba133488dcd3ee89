#!/bin/bash
# r5ad: the multi-frame statistics' chain wave with two frames' chains per lane (ILP2; with masked write-back too):
# bit-exactness, the kernel alone, the c5 200 kHz line
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
D=sdr-for-android-lib_amd/lib
for v in ilp2 ilp2wm; do
  SDRG_LIB_PATH=$D/libsdrg_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_stats_geometry.py tests/test_gpu_stats_exact.py tests/test_gpu_parity.py > gpurun_out/r5ad_tests_$v.log 2>&1 || { echo "tests FAILED on $v"; tail -20 gpurun_out/r5ad_tests_$v.log; exit 1; }
  echo "tests $v: $(tail -1 gpurun_out/r5ad_tests_$v.log)"
done
for i in 1 2; do
  for v in base ilp2 ilp2wm; do
    L=$D/libsdrg_$v.so; [ $v == base ] && L=$D/libsdrg.so
    echo "$v: $(SDRG_LIB_PATH=$L timeout -k 10 120 python tools/lab/stats_time.py 65536 200 1024 30 2>/dev/null | tail -1)"
  done
done
bash tools/ab.sh -r 2 -o c5i base ilp2 ilp2wm -- python bench.py --config c5 --focus 200 --steps 100 --warmup 20 --no-cpu-baseline
