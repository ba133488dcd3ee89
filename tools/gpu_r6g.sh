#!/bin/bash
# r6g: the low-pass outputs through a global ring (lab "gstore", SDRG_LPF_GSTORE=1): SSB parity, the SSB stage's stamps
# against the product source (lab "lab"), the c3 line alternating; then the low-pass I/O microbenchmark's write forms.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=sdr-for-android-lib_amd/lib
SDRG_LIB_PATH=$L/libsdrg_gstore.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_pulse.py tests/test_gpu_ssb_schedule.py tests/test_gpu_ssb_variant.py tests/test_gpu_edges.py \
  > gpurun_out/r6g_tests_gstore.log 2>&1 || { echo "gstore tests FAILED"; tail -40 gpurun_out/r6g_tests_gstore.log; exit 1; }
echo "gstore: $(tail -1 gpurun_out/r6g_tests_gstore.log)"
for v in lab gstore lab gstore; do
  SDRG_LIB_PATH=$L/libsdrg_$v.so SDRG_PIPE_STAMPS=1 timeout -k 10 200 python tools/lab/step_once.py ${v}_ssb 4 > gpurun_out/r6g_stamps_${v}_ssb.log 2>&1 || { echo "stamps $v failed"; tail gpurun_out/r6g_stamps_${v}_ssb.log; exit 1; }
  echo "$v: $(grep 'wave 1 LPF' gpurun_out/r6g_stamps_${v}_ssb.log | tail -1 | sed 's/.*steady/steady/') | $(grep ms/step gpurun_out/r6g_stamps_${v}_ssb.log)"
done
grep -v "abs entry" gpurun_out/r6g_stamps_gstore_ssb.log | tail -13
tools/ab.sh -r 2 -o r6g base gstore -- python bench.py --steps 200 --warmup 100 --no-cpu-baseline --no-labelled || exit 1
timeout -k 10 120 ./tools/lab/lpf_io
