#!/bin/bash
# four-step wave size (frames per A/B launch pair; the scratch is 512 KiB per frame) for BASELINE configs[4]
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/sdr-for-android-lib_amd/lib
run() {
  lib=""; [ "$1" != product ] && lib=$L/libsdrg_$1.so
  SDRG_LIB_PATH=$lib timeout -k 10 200 python bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-labelled --config c5 --focus 5 > gpurun_out/wv_$1_$2.json 2> gpurun_out/wv_$1_$2.err || { echo "bench $1 failed"; tail -5 gpurun_out/wv_$1_$2.err; exit 1; }
  echo "$1 $2 $(tail -1 gpurun_out/wv_$1_$2.json | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["kernel_ms"])')"
}
for r in a b; do run product $r && run w192 $r && run w256 $r && run w320 $r && run w384 $r || exit 1; done
