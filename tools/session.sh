#!/bin/bash
# r5bh: SSB workgroup start skew with the c3 step's statistics asynchronous (mode 6), on the main stream (mode 2), and
# asynchronous with the SSB stream at high priority (SDRG_STREAM_PRIO=0,-1); then the c3 line A/B for that priority
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
L=$PWD/sdr-for-android-lib_amd/lib/libsdrg_labt.so
for v in "6 -" "2 -" "6 0,-1"; do
  set -- $v
  m=$1; pr=$2; tag=m${m}_${pr/,/_}
  if [ "$pr" == "-" ]; then unset SDRG_STREAM_PRIO; else export SDRG_STREAM_PRIO=$pr; fi
  LAB_ALL_ONLY=1 LAB_PIPE_MODE=$m SDRG_LIB_PATH=$L SDRG_PIPE_STAMPS=1 timeout -k 10 200 python3 tools/lab/coresidency_stamps.py > gpurun_out/r5bh_$tag.log 2>&1 || { tail gpurun_out/r5bh_$tag.log; exit 1; }
  echo "mode $m prio $pr:"
  awk '/^BLOCK/{b=$2; getline; next} /workgroup loop starts/{if(b) w[b]=$0} /wave 1 LPF/{if(b){print w[b]; print $0; b=""}}' gpurun_out/r5bh_$tag.log | sed 's/\[sdrg stamps\]//; s/work [0-9]* loop/loop/g' | cut -c1-220
done
unset SDRG_STREAM_PRIO
bash tools/ab.sh -r 2 -o r5bh labt "labt+p:SDRG_STREAM_PRIO=0,-1" -- python bench.py --no-cpu-baseline --no-labelled
