#!/bin/bash
# Per-role SSB cycles (stamps, SSB stage alone and the pipelined step) for the round-2 pipeline (lab r2), the 16-stream
# pipeline with the 5-slot y ring (lab pg16) and the 32-stream one (lab pg32lab, split as the product)
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/sdr-for-android-lib_amd/lib
for v in r2 pg16 pg32lab; do
  SDRG_LIB_PATH=$L/libsdrg_$v.so SDRG_PIPE_STAMPS=1 timeout -k 10 120 python bench.py --steps 2 --warmup 1 --prewarm-ms 0 --no-cpu-baseline --stages ssb > gpurun_out/st_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/st_$v.log; exit 1; }
  echo "== $v alone"; grep "sdrg stamps" gpurun_out/st_$v.log | tail -16 | cut -c15-80
  SDRG_LIB_PATH=$L/libsdrg_$v.so timeout -k 10 120 python bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-labelled > gpurun_out/stb_$v.json 2> gpurun_out/stb_$v.err || { echo "$v bench failed"; exit 1; }
  echo "$v $(tail -1 gpurun_out/stb_$v.json | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["kernel_ms"], d["ssb_latency_floor"]["ssb_ms_alone"])')"
done
