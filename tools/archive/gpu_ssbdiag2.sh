#!/bin/bash
# which co-scheduled roles slow the critical LPF wave: skip one role at a time (timing only, wrong PCM)
export TMPDIR=/tmp
run() { SDRG_PIPE_STAMPS=1 SDRG_PIPE_SKIP=$1 timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --stages ssb > gpurun_out/ssbdiag.log 2>&1 || exit 1; echo "== skip $1 $2: $(grep stamps gpurun_out/ssbdiag.log | tail -12 | awk '$5=="LPF" {printf "LPF work %s loop %s", $7, $10}')"; }
run 0 "none"
run 0x200 "DES-1"
run 0x040 "EQ"
run 0x240 "DES-1 + EQ"
run 0x001 "DC"
run 0x004 "AGC"
run 0xF00 "all DES"
run 0x0B0 "FIR-0 FIR-1 OUT"
