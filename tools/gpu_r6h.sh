#!/bin/bash
# r6h: the low-pass loop with its VALU on 64 lanes and its LDS operations on 16 (lab "split", SDRG_LPF_SPLIT=1) beside
# the four-copies form ("copies"): the lab loop on one CU and on the whole chip, SSB parity, in-situ stamps (and the
# copies form with helper roles skipped), then the c3 line alternating.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=sdr-for-android-lib_amd/lib
timeout -k 10 120 ./tools/lab/lpf_loop_lab || exit 1
SDRG_LIB_PATH=$L/libsdrg_split.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_pulse.py tests/test_gpu_ssb_schedule.py \
  > gpurun_out/r6h_tests_split.log 2>&1 || { echo "split tests FAILED"; tail -40 gpurun_out/r6h_tests_split.log; exit 1; }
echo "split: $(tail -1 gpurun_out/r6h_tests_split.log)"
for spec in lab:0 split:0 copies:0 copies:0x90 copies:0xF00 copies:0x8 copies:0xFFD split:0xFFD lab:0; do
  v=${spec%%:*}; m=${spec#*:}
  SDRG_LIB_PATH=$L/libsdrg_$v.so SDRG_PIPE_STAMPS=1 SDRG_PIPE_SKIP=$m timeout -k 10 200 python tools/lab/step_once.py ${v}_$m 4 > gpurun_out/r6h_stamps_${v}_$m.log 2>&1 || { echo "stamps $spec failed"; tail gpurun_out/r6h_stamps_${v}_$m.log; exit 1; }
  echo "$spec: $(grep 'wave 1 LPF' gpurun_out/r6h_stamps_${v}_$m.log | tail -1 | sed 's/.*steady/steady/') | $(grep ms/step gpurun_out/r6h_stamps_${v}_$m.log)"
done
tools/ab.sh -r 2 -o r6h base split copies -- python bench.py --steps 200 --warmup 100 --no-cpu-baseline --no-labelled
