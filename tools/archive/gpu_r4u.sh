#!/bin/bash
# round 4 HEAD: bench.py's N > 1 path rehearsed on the one GPU (2 gloo ranks), the one-rank RCCL group line
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_rehearse.sh || exit 1
timeout -k 10 300 python bench.py --process-group --steps 50 --warmup 5 --no-labelled --no-cpu-baseline > gpurun_out/r4u_pg.json 2>gpurun_out/r4u_pg.err || { tail -20 gpurun_out/r4u_pg.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r4u_pg.json')); print('pg', d['value'], d['ms_per_step'], d.get('backend'), d.get('gather_check'), d.get('gather_mode'))"
