#!/bin/bash
# bench.py's self-launching N = 2 path on a one-GPU box (gloo rehearsal, both ranks on cuda:0), with the spectra gather
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 2 --rehearse-gloo --streams 1024 --no-cpu-baseline > gpurun_out/rehearse2.log 2>&1 || { echo "rehearsal failed"; tail -30 gpurun_out/rehearse2.log; exit 1; }
grep '"metric"' gpurun_out/rehearse2.log | python3 -c "
import sys, json; d = json.loads(sys.stdin.read()); print(d['n_gpus'], d['value'], d.get('ranks_seen'), d.get('backend'), d.get('rehearsal_check'), d.get('spectra_gather'))"
