#!/bin/bash
# The current GPU session's steps (overwritten per session; git history keeps each one).  Run: gpurun -- bash tools/session.sh
# r5a: the C-ABI RCCL gather, the profiling-pause timing fix, the labelled lines'
# per-kernel times, then the default bench line and the one-rank --process-group line through the C ABI.
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
T=r5a
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_dist_capi.py \
  tests/test_gpu_engine_api.py tests/test_gpu_rccl.py > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -3 gpurun_out/${T}_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
python3 tools/bench_summary.py gpurun_out/${T}_bench.json
for i in 1 2; do
  timeout -k 10 200 python bench.py --process-group --steps 200 --warmup 100 --no-cpu-baseline --no-labelled > gpurun_out/${T}_pg$i.json 2> gpurun_out/${T}_pg$i.err || { tail -20 gpurun_out/${T}_pg$i.err; exit 1; }
  timeout -k 10 200 python bench.py --steps 200 --warmup 100 --no-cpu-baseline --no-labelled > gpurun_out/${T}_nopg$i.json 2> gpurun_out/${T}_nopg$i.err || { tail -20 gpurun_out/${T}_nopg$i.err; exit 1; }
  python3 -c "
import json
a=json.load(open('gpurun_out/${T}_pg$i.json')); b=json.load(open('gpurun_out/${T}_nopg$i.json'))
print('pg', a['value'], a['ms_per_step'], a.get('backend'), a.get('gather_check'), a.get('rccl_version'), '| no pg', b['value'], b['ms_per_step'])"
done
bash tools/gpu_rehearse.sh > gpurun_out/${T}_rehearse.log 2>&1; echo "rehearse exit $?"; tail -5 gpurun_out/${T}_rehearse.log
