#!/bin/bash
# round 4: the narrow statistics kernel at <= 64 VGPRs (n64: one wave per SIMD fits beside the persistent spectrum
# kernel's four) against the product (nbase), each with the statistics after the spectrum (sync) or beside the next
# call's spectrum (async): the c3 and configs[1] lines, alternating
export TMPDIR=/tmp
mkdir -p gpurun_out
D=sdr-for-android-lib_amd/lib
SDRG_LIB_PATH=$D/libsdrg_n64b8.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_stats_geometry.py > gpurun_out/r4n_tests.log 2>&1 || { tail -20 gpurun_out/r4n_tests.log; exit 1; }
echo "n64 tests: $(tail -1 gpurun_out/r4n_tests.log)"
for i in 1 2; do
  for v in nbase n64 n64b8; do
    echo "$v narrow alone: $(SDRG_LIB_PATH=$D/libsdrg_$v.so timeout -k 10 60 python tools/lab/stats_time.py 16384 5 4096 30)" || exit 1
    for a in 0 1; do
      SDRG_LIB_PATH=$D/libsdrg_$v.so timeout -k 10 200 python bench.py --steps 200 --warmup 20 --stats-async $a > gpurun_out/r4n.json 2>/dev/null || exit 1
      echo "$v async=$a $(python3 -c "import json; d=json.load(open('gpurun_out/r4n.json')); l=d['labelled']; print('c3', d['value'], d['ms_per_step'], 'c1', l['configs1_fft_stats']['value'], l['configs1_fft_stats']['ms_per_step'])")"
    done
  done
done
