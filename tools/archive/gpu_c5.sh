#!/bin/bash
# four-step (N = 65536) kernel times: product library vs a lab variant ($1), plus parity of the product
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/st.log 2>&1 || { tail -20 gpurun_out/st.log; exit 1; }
tail -1 gpurun_out/st.log
for L in "" sdr-for-android-lib_amd/lib/libsdrg_$1.so; do
  SDRG_LIB_PATH=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/c5p -o run --output-format csv -- python3 bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/c5p.log 2>&1 || exit 1
  echo "lib=${L:-product} $(grep -o '"value": [0-9.]*' gpurun_out/c5p.log)"
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/c5p/run_kernel_stats.csv')):
    if 'four' in r['Name']: print('  ', r['Name'][36:60], r['Calls'], float(r['AverageNs'])/1e3)"
done
