#!/bin/bash
# which phase of spectrum16k_kernel makes the LDS bank conflicts: ablation builds under one PMC pass each
export TMPDIR=/tmp
mkdir -p gpurun_out
for b in fftlab fftlab_pm1 fftlab_pm2 fftlab_pm4; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES -d gpurun_out/ldsc_$b -o run --output-format csv -- ./tools/fftlab/$b 4096 k16 > gpurun_out/ldsc_$b.log 2>&1 || { echo "$b failed"; tail -3 gpurun_out/ldsc_$b.log; exit 1; }
  echo "$b ok"
done
