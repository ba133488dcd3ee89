#!/bin/bash
# round 4: the new tests first (RCCL one-rank group, ADVICE fixes), then the whole GPU suite + smoke, then the
# default bench line and the one-rank RCCL rehearsal line (bench.py --process-group)
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r4a}
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_rccl.py \
    tests/test_gpu_engine_api.py tests/test_gpu_ssb_processor.py > gpurun_out/${T}_new.log 2>&1 || { tail -30 gpurun_out/${T}_new.log; exit 1; }
grep -E "passed|failed" gpurun_out/${T}_new.log | tail -1
bash tools/gpu_tests_all.sh || exit 1
cp gpurun_out/gpu_tests.log gpurun_out/${T}_gpu_tests.log
timeout -k 10 300 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
timeout -k 10 200 python bench.py --process-group --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/${T}_pg.json 2> gpurun_out/${T}_pg.err || { tail -20 gpurun_out/${T}_pg.err; exit 1; }
python3 - <<PY
import json
d = json.load(open("gpurun_out/${T}_bench.json"))
print("bench", d["value"], d["ms_per_step"], d["kernel_ms"], d["ssb_latency_floor"], d.get("roofline_dominant", {}).get("frac"))
p = json.load(open("gpurun_out/${T}_pg.json"))
print("pg", p["value"], p["ms_per_step"], p.get("backend"), p.get("ranks_seen"), p.get("gather_check"), p.get("spectra_gather"))
PY
