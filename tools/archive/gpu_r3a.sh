#!/bin/bash
# Product (16-stream pipeline, generalised) against the round-2 pipeline (lab r2), alternating; then the round profile.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ssb_schedule.py tests/test_gpu_parity.py tests/test_gpu_ssb_variant.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3a_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r3a_tests.log; exit 1; }
tail -1 gpurun_out/r3a_tests.log
L=$PWD/sdr-for-android-lib_amd/lib
run() {  # label lib
  SDRG_LIB_PATH=$2 timeout -k 10 200 python bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-labelled > gpurun_out/r3a_$1.json 2> gpurun_out/r3a_$1.err || { echo "bench $1 failed"; tail -5 gpurun_out/r3a_$1.err; exit 1; }
  echo "$1 $(tail -1 gpurun_out/r3a_$1.json | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["kernel_ms"], d["ssb_latency_floor"]["ssb_ms_alone"], d["roofline_isolated"]["frac"])')"
}
run product "" && run r2 $L/libsdrg_r2.so && run product_b "" && run r2_b $L/libsdrg_r2.so || exit 1
bash tools/profile_round.sh r3a
