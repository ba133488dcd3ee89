#!/bin/bash
# LPF chain variants: per-role work/loop cycles (stamps) and the ssb kernel time, product vs lab builds
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { SDRG_LIB_PATH=$3 SDRG_PIPE_STAMPS=1 SDRG_PIPE_SKIP=$1 timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --stages ssb > gpurun_out/lpfvar.log 2>&1 || exit 1; echo "== $2 skip $1"; grep stamps gpurun_out/lpfvar.log | tail -12 | awk '{printf "%s:%s/%s ", $5, $7, $10} END {print ""}'; }
for L in "" sdr-for-android-lib_amd/lib/libsdrg_$1.so; do
  run 0 "lib=${L:-product}" $L
  run 0xF04 "lib=${L:-product}" $L
  SDRG_LIB_PATH=$L timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/lpfvar_b.log 2>&1 || exit 1
  grep metric gpurun_out/lpfvar_b.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('bench', d['value'], d['kernel_ms'])"
done
