#!/bin/bash
# Serial chains with the running value as src1: GPU SSB tests, per-role stamps (lab build of the product), and the
# bench against the round-2 pipeline (lab r2) and the 32-stream split (lab pg32lab), alternating.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ssb_schedule.py tests/test_gpu_parity.py tests/test_gpu_ssb_variant.py tests/test_gpu_edges.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3b_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r3b_tests.log; exit 1; }
tail -1 gpurun_out/r3b_tests.log
L=$PWD/sdr-for-android-lib_amd/lib
for v in prodlab pg32lab; do
  SDRG_LIB_PATH=$L/libsdrg_$v.so SDRG_PIPE_STAMPS=1 timeout -k 10 120 python bench.py --steps 2 --warmup 1 --prewarm-ms 0 --no-cpu-baseline --stages ssb > gpurun_out/r3b_st_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/r3b_st_$v.log; exit 1; }
  echo "== $v alone"; grep "sdrg stamps" gpurun_out/r3b_st_$v.log | tail -16 | cut -c15-80
done
run() {  # label lib
  SDRG_LIB_PATH=$2 timeout -k 10 200 python bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-labelled > gpurun_out/r3b_$1.json 2> gpurun_out/r3b_$1.err || { echo "bench $1 failed"; tail -5 gpurun_out/r3b_$1.err; exit 1; }
  echo "$1 $(tail -1 gpurun_out/r3b_$1.json | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["kernel_ms"], d["ssb_latency_floor"]["ssb_ms_alone"], d["roofline_isolated"]["frac"])')"
}
run product "" && run r2 $L/libsdrg_r2.so && run pg32 $L/libsdrg_pg32lab.so && run product_b "" && run r2_b $L/libsdrg_r2.so
