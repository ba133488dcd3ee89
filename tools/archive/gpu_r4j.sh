#!/bin/bash
# round 4: the spectrum kernel's leaner tail (SDRG_K16_V2: scale folded into the pass-2 twiddles, unpacked |X|^2 without
# pair transposes, buffer stores, no zeroing branch) against the round-3 tail: fftlab alone (bits hash, alternating),
# GPU parity tests on the product library, then the default and configs[1] lines A/B on the lab builds
export TMPDIR=/tmp
mkdir -p gpurun_out
D=sdr-for-android-lib_amd/lib
for i in 1 2 3; do
  for b in fftlab_v1 fftlab_v2; do echo "$b: $(timeout -k 5 60 tools/fftlab/$b 4096 k16)" || exit 1; done
done > gpurun_out/r4j_fftlab.log 2>&1 || { cat gpurun_out/r4j_fftlab.log; exit 1; }
cat gpurun_out/r4j_fftlab.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_any_n.py tests/test_gpu_e2e_exposure.py > gpurun_out/r4j_tests.log 2>&1 || { tail -30 gpurun_out/r4j_tests.log; exit 1; }
tail -3 gpurun_out/r4j_tests.log
cat gpurun_out/e2e_exposure.json | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['total'])"
for i in 1 2; do
  for v in k16v1 k16v2; do
    SDRG_LIB_PATH=$D/libsdrg_$v.so timeout -k 10 200 python bench.py --steps 200 --warmup 20 > gpurun_out/r4j.json 2>/dev/null || exit 1
    echo "$v c3 $(python3 -c "import json; d=json.load(open('gpurun_out/r4j.json')); print(d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline_isolated']['achieved'], d['labelled']['configs1_fft_stats']['value'])")"
  done
done
