#!/bin/bash
# r6v: the driver's bench command after the labelled lines' step floor (LABELLED_MIN_STEPS)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6v_driverlike.json 2> gpurun_out/r6v_driverlike.err || { echo "bench failed"; tail gpurun_out/r6v_driverlike.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r6v_driverlike.json").read().strip().splitlines()[-1])
print("driver", d["value"], d["ms_per_step"])
for k, v in d["labelled"].items():
    print(k, v["value"], v["ms_per_step"], v.get("steps"))
PY
