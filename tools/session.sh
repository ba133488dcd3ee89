#!/bin/bash
# r5az: FFT + statistics (BASELINE configs[1], bench --config c2) with the asynchronous statistics on a CU partition of
# their own (lab SDRG_STATS_CUS = k CUs, the spectrum on the others) against the one-stream schedule, alternating
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
L=sdr-for-android-lib_amd/lib/libsdrg_labs.so
run() {  # label env... -- args
  local tag=$1; shift
  env SDRG_LIB_PATH=$L "$@" > gpurun_out/r5az_$tag.json 2> gpurun_out/r5az_$tag.err || { echo "$tag failed"; tail -5 gpurun_out/r5az_$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernel_ms']; print(sys.argv[2], round(d['value']/1e3,1), 'G', d['ms_per_step'], 'ms spec', k.get('spectrum_ms'), 'stats', k.get('stats_ms'))" gpurun_out/r5az_$tag.json $tag
}
for r in 1 2; do
  run one_$r timeout -k 10 200 python bench.py --config c2 --no-cpu-baseline --no-labelled
  run async_$r timeout -k 10 200 python bench.py --config c2 --stats-async 1 --no-cpu-baseline --no-labelled
  for k in 16 32 64; do
    run k${k}_$r env SDRG_STATS_CUS=$k timeout -k 10 200 python bench.py --config c2 --stats-async 1 --no-cpu-baseline --no-labelled
  done
done
