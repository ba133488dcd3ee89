#!/bin/bash
# pipelined bench under stream priorities (SDRG_STREAM_PRIO=main,ssb; lower = higher priority)
export TMPDIR=/tmp
python - <<'PY'
import ctypes
h = ctypes.CDLL("libamdhip64.so")
lo, hi = ctypes.c_int(), ctypes.c_int()
h.hipDeviceGetStreamPriorityRange(ctypes.byref(lo), ctypes.byref(hi))
print("priority range least", lo.value, "greatest", hi.value)
PY
for p in "0,0" "-1,0" "0,-1" "0,0"; do
  SDRG_STREAM_PRIO=$p timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/b.log 2>&1 || { tail -5 gpurun_out/b.log; exit 1; }
  echo "prio=$p $(grep metric gpurun_out/b.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['kernel_ms'])")"
done
