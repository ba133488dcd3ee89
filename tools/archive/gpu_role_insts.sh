#!/bin/bash
# SSB pipeline instruction count per role: SQ_INSTS_VALU / LDS / SALU of the SSB stage alone with each role's
# work skipped in turn (SDRG_PIPE_SKIP, diagnostic: wrong results); role r's count = all - skipped(r)
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
for r in none 0 1 2 3 4 5 6 7 8 9 10 11; do
  if [ $r = none ]; then m=0; else m=$((1 << r)); fi
  cd /tmp && SDRG_PIPE_SKIP=$m timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES -d $R/gpurun_out/roles_$r -o run --output-format csv -- python3 $R/tools/kernel_lab.py --stages ssb --calls 3 > $R/gpurun_out/roles_$r.log 2>&1 || { echo "role $r failed"; tail -3 $R/gpurun_out/roles_$r.log; exit 1; }
  cd $R
done
echo done
