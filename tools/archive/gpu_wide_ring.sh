#!/bin/bash
# configs[4] at 200 kHz: a smaller wide-statistics LDS ring (SDRG_WIDE_RING 4608 / 6144 floats instead of 9216), so the
# four-step FFT kernels of the next call fit beside the statistics workgroups; ring24 also with the persistent
# four-step kernels.  ring18 is benched at 200 kHz only (three windows; its ring is too small for 11-window geometries).
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/sdr-for-android-lib_amd/lib
for v in ring24 ring24fp; do SDRG_LIB_PATH=$L/libsdrg_$v.so timeout -k 10 200 python -u -m pytest tests/test_gpu_stats_exact.py tests/test_gpu_stats_geometry.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "200 or 65536" > gpurun_out/wr_tests_$v.log 2>&1 || { echo "tests $v failed"; tail -20 gpurun_out/wr_tests_$v.log; exit 1; }; tail -n 1 gpurun_out/wr_tests_$v.log; done
run() {
  lib=""; [ "$1" != product ] && lib=$L/libsdrg_$1.so
  SDRG_LIB_PATH=$lib timeout -k 10 200 python bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-labelled --config c5 --focus $3 > gpurun_out/wr_$1_$2_$3.json 2> gpurun_out/wr_$1_$2_$3.err || { echo "bench $1 failed"; tail -5 gpurun_out/wr_$1_$2_$3.err; exit 1; }
  echo "$1 $2 focus $3: $(tail -n 1 gpurun_out/wr_$1_$2_$3.json | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["kernel_ms"])')"
}
for r in a b; do run product $r 200 && run ring18 $r 200 && run ring24 $r 200 && run ring24fp $r 200 || exit 1; done
run ring24fp a 5 && run product c 5 || exit 1
