#!/bin/bash
# r5ah: the 65536-point four-step in two streams (column kernel of wave w + 1 beside the row kernel of wave w, two
# intermediate buffers): parity, the FFT alone, the configs[4] lines
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
D=sdr-for-android-lib_amd/lib
for v in fs2s fs2s96; do
  SDRG_LIB_PATH=$D/libsdrg_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_any_n.py tests/test_gpu_stats_geometry.py > gpurun_out/r5ah_tests_$v.log 2>&1 || { echo "tests FAILED on $v"; tail -20 gpurun_out/r5ah_tests_$v.log; exit 1; }
  echo "tests $v: $(tail -1 gpurun_out/r5ah_tests_$v.log)"
done
for i in 1 2; do
  for v in base fs2s fs2s96; do
    L=$D/libsdrg_$v.so; [ $v == base ] && L=$D/libsdrg.so
    echo "$v: $(SDRG_LIB_PATH=$L timeout -k 10 120 python tools/lab/spec_time.py 65536 cs16 1024 50 2>&1 | tail -1)"
  done
done
bash tools/ab.sh -r 2 -o c5a base fs2s fs2s96 -- python bench.py --config c5 --focus 5 --steps 100 --warmup 20 --no-cpu-baseline
bash tools/ab.sh -r 1 -o c5b base fs2s fs2s96 -- python bench.py --config c5 --focus 200 --steps 100 --warmup 20 --no-cpu-baseline
