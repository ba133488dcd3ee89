#!/bin/bash
# s_setprio masks of the SSB pipeline roles (SDRG_PIPE_PRIO): per-role stamps and the ssb kernel time
export TMPDIR=/tmp
mkdir -p gpurun_out
for P in 0x7 0x0 0x2 0x6 0xF00; do
  SDRG_PIPE_PRIO=$P SDRG_PIPE_STAMPS=1 timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --stages ssb > gpurun_out/prio3.log 2>&1 || exit 1
  echo "== prio $P"; grep stamps gpurun_out/prio3.log | tail -12 | awk '{printf "%s:%s/%s ", $5, $7, $10} END {print ""}'
done
