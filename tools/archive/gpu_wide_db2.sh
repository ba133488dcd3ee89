#!/bin/bash
# Wide statistics (65536 / 200 kHz): the pooled-gap pass reads the scan's dB values, copied to the pool scratch by the
# record wave (SDRG_WIDE_DBPOOL=2, lab build db2): parity tests, per-phase stamps, alternating bench lines
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/sdr-for-android-lib_amd/lib
SDRG_LIB_PATH=$L/libsdrg_db2.so timeout -k 10 200 python -u -m pytest tests/test_gpu_stats_exact.py tests/test_gpu_stats_geometry.py tests/test_gpu_parity.py tests/test_gpu_any_n.py -m gpu -x -q --timeout 120 --timeout-method thread -k "200 or 65536 or 131072 or 786432 or 1048576" > gpurun_out/db2_tests.log 2>&1 || { echo "tests db2 failed"; tail -20 gpurun_out/db2_tests.log; exit 1; }
tail -n 1 gpurun_out/db2_tests.log
SDRG_LIB_PATH=$L/libsdrg_stamps_db2.so timeout -k 10 120 python tools/kernel_lab.py --stages spectrum+stats --n 65536 --fmt CS16 --streams 1024 --focus 200 --calls 3 > gpurun_out/db2_st.log 2>&1 || { echo "stamps failed"; tail gpurun_out/db2_st.log; exit 1; }
grep -v amdgpu.ids gpurun_out/db2_st.log
run() {
  lib=""; [ "$1" != product ] && lib=$L/libsdrg_$1.so
  SDRG_LIB_PATH=$lib timeout -k 10 200 python bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-labelled --config c5 --focus 200 > gpurun_out/db2_$1_$2.json 2> gpurun_out/db2_$1_$2.err || { echo "bench $1 failed"; tail -5 gpurun_out/db2_$1_$2.err; exit 1; }
  echo "$1 $2: $(tail -n 1 gpurun_out/db2_$1_$2.json | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["kernel_ms"])')"
}
for r in a b; do run product $r && run db2 $r || exit 1; done
