#!/bin/bash
# r6j: the low-pass loop with full-EXEC VALU, 16-lane LDS reads and global-store outputs (lab "sgs": SDRG_LPF_SPLIT=1 +
# SDRG_LPF_GSTORE=1): SSB parity, in-situ stamps (all roles, and every other role skipped), c3 line alternating.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=sdr-for-android-lib_amd/lib
SDRG_LIB_PATH=$L/libsdrg_sgs.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_pulse.py tests/test_gpu_ssb_schedule.py tests/test_gpu_ssb_variant.py tests/test_gpu_edges.py \
  > gpurun_out/r6j_tests_sgs.log 2>&1 || { echo "sgs tests FAILED"; tail -40 gpurun_out/r6j_tests_sgs.log; exit 1; }
echo "sgs: $(tail -1 gpurun_out/r6j_tests_sgs.log)"
for spec in lab:0 sgs:0 sgs:0xFFD gstore:0 copies:0 sgs:0 lab:0; do
  v=${spec%%:*}; m=${spec#*:}
  SDRG_LIB_PATH=$L/libsdrg_$v.so SDRG_PIPE_STAMPS=1 SDRG_PIPE_SKIP=$m timeout -k 10 200 python tools/lab/step_once.py ${v}_$m 4 > gpurun_out/r6j_stamps_${v}_$m.log 2>&1 || { echo "stamps $spec failed"; tail gpurun_out/r6j_stamps_${v}_$m.log; exit 1; }
  echo "$spec: $(grep 'wave 1 LPF' gpurun_out/r6j_stamps_${v}_$m.log | tail -1 | sed 's/.*steady/steady/') | $(grep ms/step gpurun_out/r6j_stamps_${v}_$m.log)"
done
tools/ab.sh -r 2 -o r6j base sgs -- python bench.py --steps 200 --warmup 100 --no-cpu-baseline --no-labelled
