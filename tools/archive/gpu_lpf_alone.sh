#!/bin/bash
# SSB loop cycles with every role, with the low-pass wave alone (others skipped) and with the low-pass wave skipped
export TMPDIR=/tmp
mkdir -p gpurun_out
for skip in 0 0xFFD 0x2; do
  SDRG_PIPE_STAMPS=1 SDRG_PIPE_SKIP=$skip timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --stages ssb > gpurun_out/lpfa.log 2>&1 || exit 1
  echo "skip=$skip $(grep stamps gpurun_out/lpfa.log | tail -12 | awk '{w[NR]=$5":"int($8/1000)} END {for (i=1;i<=12;i++) printf "%s ", w[i]}') loop:$(grep stamps gpurun_out/lpfa.log | tail -1 | awk '{print int($10/1000)}')"
done
