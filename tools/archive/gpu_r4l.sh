#!/bin/bash
# round 4: the statistics' dB through log10f_sel (glibc's log10f, special cases by selects, no branch) against the
# branch form (log10f_fast): exhaustive device libm test, statistics GPU tests on the product, the statistics kernels
# alone (c5 200 kHz wide multi-frame, c3 narrow) and the bench lines, alternating lab builds (logfast / logsel)
export TMPDIR=/tmp
mkdir -p gpurun_out
D=sdr-for-android-lib_amd/lib
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_libm_exact.py tests/test_gpu_stats_exact.py tests/test_gpu_stats_geometry.py tests/test_gpu_parity.py > gpurun_out/r4l_tests.log 2>&1 || { tail -30 gpurun_out/r4l_tests.log; exit 1; }
tail -2 gpurun_out/r4l_tests.log
for i in 1 2; do
  for v in logfast logsel; do
    echo "$v c5/200 alone: $(SDRG_LIB_PATH=$D/libsdrg_$v.so timeout -k 10 60 python tools/lab/stats_time.py 65536 200 1024 30)" || exit 1
    echo "$v c3 narrow alone: $(SDRG_LIB_PATH=$D/libsdrg_$v.so timeout -k 10 60 python tools/lab/stats_time.py 16384 5 4096 30)" || exit 1
  done
done
for i in 1 2; do
  for v in logfast logsel; do
    SDRG_LIB_PATH=$D/libsdrg_$v.so timeout -k 10 200 python bench.py --steps 200 --warmup 20 > gpurun_out/r4l.json 2>/dev/null || exit 1
    echo "$v $(python3 -c "import json; d=json.load(open('gpurun_out/r4l.json')); l=d['labelled']; print('c3', d['value'], d['ms_per_step'], d['kernel_ms']['stats_ms'], 'c1', l['configs1_fft_stats']['value'], 'c5/5', l['configs4_c5_5khz']['value'], 'c5/200', l['configs4_c5_200khz']['value'], l['configs4_c5_200khz']['stats_ms'])")"
  done
done
