#!/bin/bash
# r6c = r6a + r6b in one call: (1) SSB parity on the barrier-free pipeline (lab "flags", SDRG_PIPE_FLAGS=1); (2) spectrum
# parity on the product (exchange trim, SDRG_K16_XCH_TRIM=1); (3) the spectrum alone, same-bits hash and time, trim vs
# round 5's exchanges (lab "xch0"); (4) the c3 line alternating: product / flags / xch0; (5) per-role stamps, barrier
# (lab "lab") vs counters (lab "flags").
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=sdr-for-android-lib_amd/lib
SDRG_LIB_PATH=$L/libsdrg_flags.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_pulse.py tests/test_gpu_ssb_schedule.py tests/test_gpu_ssb_variant.py \
  > gpurun_out/r6c_tests_flags.log 2>&1 || { echo "flags tests FAILED"; tail -40 gpurun_out/r6c_tests_flags.log; exit 1; }
echo "flags: $(tail -1 gpurun_out/r6c_tests_flags.log)"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_any_n.py tests/test_gpu_edges.py \
  > gpurun_out/r6c_tests_spec.log 2>&1 || { echo "spectrum tests FAILED"; tail -40 gpurun_out/r6c_tests_spec.log; exit 1; }
echo "product spectrum: $(tail -1 gpurun_out/r6c_tests_spec.log)"
for fmt in cs8 cs16 cu8 cf32; do
  for v in xch0 product xch0 product; do
    if [ $v = product ]; then lib=$L/libsdrg.so; else lib=$L/libsdrg_$v.so; fi
    SDRG_LIB_PATH=$lib timeout -k 10 120 python tools/lab/spec_time.py 16384 $fmt 4096 200 || exit 1
  done
done
tools/ab.sh -r 2 -o r6c base flags xch0 -- python bench.py --steps 200 --warmup 100 --no-cpu-baseline || exit 1
for v in lab flags; do
  SDRG_LIB_PATH=$L/libsdrg_$v.so SDRG_PIPE_STAMPS=1 timeout -k 10 200 python tools/lab/step_once.py $v 31 > gpurun_out/r6c_stamps_$v.log 2>&1 || { echo "stamps $v failed"; tail gpurun_out/r6c_stamps_$v.log; exit 1; }
  SDRG_LIB_PATH=$L/libsdrg_$v.so SDRG_PIPE_STAMPS=1 timeout -k 10 200 python tools/lab/step_once.py ${v}_ssb 4 > gpurun_out/r6c_stamps_${v}_ssb.log 2>&1 || { echo "stamps $v ssb failed"; exit 1; }
  grep -v "abs entry" gpurun_out/r6c_stamps_$v.log | tail -15
  grep -v "abs entry" gpurun_out/r6c_stamps_${v}_ssb.log | tail -15
done
