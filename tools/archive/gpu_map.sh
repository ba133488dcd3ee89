#!/bin/bash
# SSB pipeline under different role->wave maps (diagnostic): ms/step (ssb only, all) and stamps per map
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo "build failed"; exit 1; }
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for m in ${MAPS}; do
  SDRG_PIPE_MAP=$m timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --stages ssb > gpurun_out/map_$m.log 2>&1 || { echo "bench $m failed"; exit 1; }
  SDRG_PIPE_MAP=$m timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/mapall_$m.log 2>&1 || { echo "bench all $m failed"; exit 1; }
  SDRG_PIPE_MAP=$m SDRG_PIPE_STAMPS=1 timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --stages ssb > gpurun_out/map_stamps_$m.log 2>&1 || { echo "stamps $m failed"; exit 1; }
  echo "map $m: ssb $(grep -h ms_per_step gpurun_out/map_$m.log | python3 -c 'import sys,json; print(json.loads(sys.stdin.read())["ms_per_step"])') all $(grep -h ms_per_step gpurun_out/mapall_$m.log | python3 -c 'import sys,json; print(json.loads(sys.stdin.read())["ms_per_step"])')"
  grep "sdrg stamps" gpurun_out/map_stamps_$m.log | awk '{printf "  %s:%d", $5, $7/1000} END {print ""}'
done
