#!/bin/bash
# r6p: the low-pass wave alone on its SIMD (lab build hw15: 15 hardware waves, waves 5, 9, 13 idle; EQ and DES1
# moved to SIMDs 0 and 2) against the product map: SSB tests (bit-exact), stamps, c3 A/B.  The lab option the hw15
# build used (SDRG_PIPE_HW_WAVES, ssb.hip) was removed after the run; results in profiles/r6nop_lpf_simd.md
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=sdr-for-android-lib_amd/lib
M15=9F67BF84AF53210
for v in "lab:" "hw15:SDRG_PIPE_MAP=$M15"; do
  n=${v%%:*}; kv=${v#*:}
  for st in 4 31; do
    env SDRG_LIB_PATH=$L/libsdrg_$n.so SDRG_PIPE_STAMPS=1 $kv timeout -k 10 200 python tools/lab/step_once.py ${n}_$st $st > gpurun_out/r6p_${n}_$st.log 2>&1 || { echo "stamps $n/$st failed"; tail gpurun_out/r6p_${n}_$st.log; exit 1; }
    echo "== $n stages $st"; grep -v "abs entry" gpurun_out/r6p_${n}_$st.log | grep -E "wave|ms/step" | sed 's/last:.*steady/steady/' | tail -13
  done
done
bash tools/ab.sh -r 2 -o r6p -t "tests/test_gpu_ssb_schedule.py tests/test_gpu_ssb_processor.py tests/test_gpu_ssb_variant.py" base "hw15:SDRG_PIPE_MAP=$M15" -- python bench.py --steps 200 --warmup 100 --no-cpu-baseline --no-labelled
