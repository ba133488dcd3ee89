#!/bin/bash
# SSB pipeline under different wave-priority masks (diagnostic): ms/step (ssb only) and stamps per mask
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo "build failed"; exit 1; }
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for m in ${MASKS:-0x7 0x0 0x2 0x6 0xff}; do
  SDRG_PIPE_PRIO=$m timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --stages ssb > gpurun_out/prio_$m.log 2>&1 || { echo "bench $m failed"; exit 1; }
  SDRG_PIPE_PRIO=$m SDRG_PIPE_STAMPS=1 timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --stages ssb > gpurun_out/prio_stamps_$m.log 2>&1 || { echo "stamps $m failed"; exit 1; }
  echo "mask $m: $(grep -h ms_per_step gpurun_out/prio_$m.log | python3 -c 'import sys,json; print(json.loads(sys.stdin.read())["ms_per_step"])')"
  grep "sdrg stamps" gpurun_out/prio_stamps_$m.log | head -8
done
timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/all.log 2>&1 && echo "all: $(grep -h ms_per_step gpurun_out/all.log | python3 -c 'import sys,json; print(json.loads(sys.stdin.read())["ms_per_step"])')"
