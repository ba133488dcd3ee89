#!/bin/bash
# In-kernel SSB stamps per role (cycles, time, effective clock): steady state of a pipelined run (co-resident with
# the spectrum) vs the SSB stage alone
export TMPDIR=/tmp
mkdir -p gpurun_out
SDRG_PIPE_STAMPS=1 timeout -k 10 120 python bench.py --steps 40 --warmup 3 --no-cpu-baseline --no-labelled > gpurun_out/stamps.log 2>&1 || { echo "stamps failed"; tail gpurun_out/stamps.log; exit 1; }
grep "DC \|LPF\|AGC\|LOAD" gpurun_out/stamps.log
