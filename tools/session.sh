#!/bin/bash
# r5d: (1) wide statistics with the pooled dB sum's reads pipelined: tests, alone vs round 4, stamps per phase;
# (2) ssb64 with the front's LDS-DMA raw ring: SSB parity tests, per-role stamps, per-kernel times
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
T=r5d
D=sdr-for-android-lib_amd/lib
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_stats_exact.py \
  tests/test_gpu_stats_geometry.py > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for i in 1 2; do
  for v in r4stats base; do
    L=$D/libsdrg_$v.so; [ $v == base ] && L=$D/libsdrg.so
    echo "$v stats alone: $(SDRG_LIB_PATH=$L timeout -k 10 120 python tools/lab/stats_time.py 65536 200 1024 30 2>/dev/null | tail -1)"
  done
done
SDRG_LIB_PATH=$D/libsdrg_mwst.so timeout -k 10 120 python tools/lab/stats_time.py 65536 200 1024 3 2>&1 | grep "mw stamps" | tail -1
SDRG_LIB_PATH=$D/libsdrg_ssb64.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_pulse.py tests/test_gpu_ssb_schedule.py > gpurun_out/${T}_ssb64_tests.log 2>&1 || { tail -40 gpurun_out/${T}_ssb64_tests.log; exit 1; }
tail -1 gpurun_out/${T}_ssb64_tests.log
SDRG_SSB64_STAMPS=1 SDRG_LIB_PATH=$D/libsdrg_ssb64.so timeout -k 10 200 python bench.py --stages ssb --steps 40 --warmup 5 --no-cpu-baseline --no-labelled --prewarm-ms 0 > gpurun_out/${T}_st.json 2> gpurun_out/${T}_st.err || { tail -5 gpurun_out/${T}_st.err; exit 1; }
grep "ssb64 stamps" gpurun_out/${T}_st.err | tail -2
SDRG_LIB_PATH=$D/libsdrg_ssb64.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof64 -o run --output-format csv -- python3 bench.py --stages ssb --steps 20 --warmup 10 --no-cpu-baseline --no-labelled > gpurun_out/${T}_prof64.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/${T}_prof64.log; exit 1; }
python3 - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/r5d_prof64/**/run_kernel_stats.csv", recursive=True):
    for r in list(csv.DictReader(open(f)))[:4]:
        print(f"{r['Name'][:70]:70s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:9.1f} us")
PY
