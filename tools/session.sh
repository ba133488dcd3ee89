#!/bin/bash
# r5al: the SSB stream's kernel boundary with and without the spectrum beside it (kernel traces)
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r5al_ssb -o run -- python3 $GRAFT_REPO_ROOT/bench.py --stages ssb --steps 50 --warmup 10 --no-labelled --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r5al_ssb.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/r5al_ssb.log; exit 1; }
echo done
