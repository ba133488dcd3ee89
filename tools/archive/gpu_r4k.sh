#!/bin/bash
# round 4: the audio pulse detector on a stream of its own (the SSB stream carries the SSB kernels alone): GPU suite on
# the product library, then the default line A/B against the previous commit's library (apold), alternating
export TMPDIR=/tmp
mkdir -p gpurun_out
D=sdr-for-android-lib_amd/lib
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4k_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r4k_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r4k_gpu_tests.log
for i in 1 2; do
  for v in apold new new:sync; do
    L=$D/libsdrg.so; X=""
    if [ $v = apold ]; then L=$D/libsdrg_apold.so; fi
    if [ $v = new:sync ]; then X="--stats-async 0"; fi
    SDRG_LIB_PATH=$L timeout -k 10 200 python bench.py --steps 200 --warmup 20 $X > gpurun_out/r4k.json 2>/dev/null || exit 1
    echo "$v c3 $(python3 -c "import json; d=json.load(open('gpurun_out/r4k.json')); l=d['labelled']; print(d['value'], d['ms_per_step'], d['kernel_ms'], d['ssb_latency_floor']['ssb_ms_coresident'], 'c1', l['configs1_fft_stats'], 'c5/200', l['configs4_c5_200khz']['value'])")"
  done
done
