#!/bin/bash
# SSB pipeline role diagnostics: stamps with subsets of roles skipped (SDRG_PIPE_SKIP = roles whose work is
# skipped; wrong PCM, timing only) and alternative role maps
export TMPDIR=/tmp
run() { SDRG_PIPE_STAMPS=1 SDRG_PIPE_SKIP=$1 timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --stages ssb > gpurun_out/ssbdiag.log 2>&1 || exit 1; echo "== skip $1 $2"; grep stamps gpurun_out/ssbdiag.log | tail -12 | awk '{printf "%s %s work %s loop %s\n", $4, $5, $7, $10}'; }
run 0 "all roles"
run 0xFFD "LPF only"
run 0xDFD "LPF + EQ"
run 0xDF9 "LPF + AGC + EQ"
run 0x0F0 "no FIR/OUT/EQ"
run 0xF00 "no DES"
