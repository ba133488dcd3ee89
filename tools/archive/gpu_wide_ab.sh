#!/bin/bash
# Wide statistics (BASELINE configs[4], 65536 / 200 kHz): role rotation across SIMDs and src1-form chain adds (lab)
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/sdr-for-android-lib_amd/lib
timeout -k 10 200 python -u -m pytest tests/test_gpu_stats_exact.py tests/test_gpu_stats_geometry.py -m gpu -x -q --timeout 120 --timeout-method thread -k "200 or 65536" > gpurun_out/wab_tests.log 2>&1 || { echo "tests failed"; tail -20 gpurun_out/wab_tests.log; exit 1; }
tail -1 gpurun_out/wab_tests.log
for v in rot src1 rotsrc1; do SDRG_LIB_PATH=$L/libsdrg_$v.so timeout -k 10 200 python -u -m pytest tests/test_gpu_stats_exact.py tests/test_gpu_stats_geometry.py -m gpu -x -q --timeout 120 --timeout-method thread -k "200 or 65536" > gpurun_out/wab_tests_$v.log 2>&1 || { echo "tests $v failed"; tail -20 gpurun_out/wab_tests_$v.log; exit 1; }; done
run() {
  lib=""; [ "$1" != product ] && lib=$L/libsdrg_$1.so
  SDRG_LIB_PATH=$lib timeout -k 10 200 python bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-labelled --config c5 --focus 200 > gpurun_out/wab_$1_$2.json 2> gpurun_out/wab_$1_$2.err || { echo "bench $1 failed"; tail -5 gpurun_out/wab_$1_$2.err; exit 1; }
  echo "$1 $2 $(tail -1 gpurun_out/wab_$1_$2.json | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["kernel_ms"])')"
}
for r in a b; do run product $r && run rot $r && run src1 $r && run rotsrc1 $r || exit 1; done
