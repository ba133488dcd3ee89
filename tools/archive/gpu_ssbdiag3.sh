#!/bin/bash
# per-role work/loop cycles with roles skipped (timing only, wrong PCM): what bounds the SSB pipeline?
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { SDRG_PIPE_STAMPS=1 SDRG_PIPE_SKIP=$1 timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --stages ssb > gpurun_out/ssbdiag_$1.log 2>&1 || exit 1; echo "== skip $1 $2"; grep stamps gpurun_out/ssbdiag_$1.log | tail -12 | awk '{printf "%s:%s/%s ", $5, $7, $10} END {print ""}'; }
run 0 "none"
run 0xF00 "all DES"
run 0x004 "AGC"
run 0xF04 "AGC + all DES"
run 0x002 "LPF"
run 0xFF9 "all but LPF and AGC"
run 0xFFD "all but LPF"
