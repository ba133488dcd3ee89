#!/bin/bash
# round 4: the main stream's markers from the spectrum / statistics kernels' own dispatches (timing origin, the marker
# after the spectrum, the end marker) against the marker packets (mkold = the previous commit): GPU suite on the
# product, then the c3 default line with its labelled configs[1] / configs[4] lines and the driver's command, alternating
export TMPDIR=/tmp
mkdir -p gpurun_out
D=sdr-for-android-lib_amd/lib
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4t_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r4t_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r4t_gpu_tests.log
for i in 1 2; do
  for v in mkold new; do
    L=$D/libsdrg.so; if [ $v = mkold ]; then L=$D/libsdrg_mkold.so; fi
    SDRG_LIB_PATH=$L timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/r4t.json 2>/dev/null || exit 1
    echo "$v $(python3 -c "import json; d=json.load(open('gpurun_out/r4t.json')); l=d['labelled']; print('c3', d['value'], d['ms_per_step'], d['kernel_ms'], 'roof', d['roofline']['frac'], 'c1', l['configs1_fft_stats']['ms_per_step'], 'c5/5', l['configs4_c5_5khz']['ms_per_step'], 'c5/200', l['configs4_c5_200khz']['ms_per_step'])")"
    SDRG_LIB_PATH=$L timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-labelled --no-cpu-baseline > gpurun_out/r4t20.json 2>/dev/null || exit 1
    echo "$v 20-step $(python3 -c "import json; d=json.load(open('gpurun_out/r4t20.json')); print(d['value'], d['ms_per_step'])")"
  done
done
