#!/bin/bash
# Wide statistics (65536 / 200 kHz): chain-wave LDS read-ahead (SDRG_WIDE_SETS 3/4 register sets) against the product
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/sdr-for-android-lib_amd/lib
for v in s3 s4; do SDRG_LIB_PATH=$L/libsdrg_$v.so timeout -k 10 200 python -u -m pytest tests/test_gpu_stats_exact.py tests/test_gpu_stats_geometry.py -m gpu -x -q --timeout 120 --timeout-method thread -k "200 or 65536" > gpurun_out/wsets_tests_$v.log 2>&1 || { echo "tests $v failed"; tail -20 gpurun_out/wsets_tests_$v.log; exit 1; }; tail -n 1 gpurun_out/wsets_tests_$v.log; done
for v in stamps stamps_s3; do SDRG_LIB_PATH=$L/libsdrg_$v.so timeout -k 10 120 python tools/kernel_lab.py --stages spectrum+stats --n 65536 --fmt CS16 --streams 1024 --focus 200 --calls 3 > gpurun_out/wsets_st_$v.log 2>&1 || { echo "stamps $v failed"; tail gpurun_out/wsets_st_$v.log; exit 1; }; echo "== $v"; grep -v amdgpu.ids gpurun_out/wsets_st_$v.log; done
run() {
  lib=""; [ "$1" != product ] && lib=$L/libsdrg_$1.so
  SDRG_LIB_PATH=$lib timeout -k 10 200 python bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-labelled --config c5 --focus 200 > gpurun_out/wsets_$1_$2.json 2> gpurun_out/wsets_$1_$2.err || { echo "bench $1 failed"; tail -5 gpurun_out/wsets_$1_$2.err; exit 1; }
  echo "$1 $2 $(tail -n 1 gpurun_out/wsets_$1_$2.json | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["kernel_ms"])')"
}
for r in a b; do run product $r && run s3 $r && run s4 $r || exit 1; done
