#!/bin/bash
# AGC sqrt from rsq + one residual step (product) vs the estimate-and-select sqrt (lab build prevsqrt): the exhaustive exactness
# test, the SSB parity tests, then alternating default bench lines
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_agc_math.py tests/test_gpu_parity.py tests/test_gpu_ssb_variant.py tests/test_gpu_ssb_processor.py tests/test_gpu_edges.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/sqrt_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/sqrt_tests.log; exit 1; }
tail -n 1 gpurun_out/sqrt_tests.log
L=$PWD/sdr-for-android-lib_amd/lib
run() {
  lib=""; [ "$1" != product ] && lib=$L/libsdrg_$1.so
  SDRG_LIB_PATH=$lib timeout -k 10 200 python bench.py --steps 300 --warmup 50 --no-cpu-baseline --no-labelled > gpurun_out/sqrt_$1_$2.json 2> gpurun_out/sqrt_$1_$2.err || { echo "bench $1 failed"; tail -5 gpurun_out/sqrt_$1_$2.err; exit 1; }
  echo "$1 $2 $(tail -n 1 gpurun_out/sqrt_$1_$2.json | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["kernel_ms"], d["ssb_latency_floor"]["ssb_ms_alone"])')"
}
for r in a b c; do run product $r && run prevsqrt $r || exit 1; done
