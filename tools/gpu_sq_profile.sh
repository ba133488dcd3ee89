#!/bin/bash
# SQ counters of the spectrum and statistics kernels (one pass per counter group, kernel-trace only, each under its
# own hard time limit): spectrum16k alone (c3/c2 size), spectrum + stats at c2 (16384, 5 kHz) and c5 (65536 CS16,
# 200 kHz), and the c3 pipeline (all stages, pipelined: the co-resident view).  -> gpurun_out/sq_<prog>_<pass>/
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-sq}
declare -A PROG
PROG[spec]="--stages spectrum --calls 10"
PROG[c2]="--stages spectrum+stats --calls 10"
PROG[c5]="--stages spectrum+stats --n 65536 --fmt CS16 --streams 1024 --focus 200 --calls 4"
PROG[c3]="--stages all --pipelined 1 --calls 12"
PROG[ssb]="--stages ssb --calls 10"
PASS_a="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU"
PASS_b="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
PASS_c="SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_STORE SQ_INSTS_LDS_ATOMIC SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
for p in ${PROGS:-spec c2 c5 c3}; do
  for pass in a b c; do
    v=PASS_$pass
    cd /tmp && timeout -s KILL 90 rocprofv3 --kernel-trace --pmc ${!v} -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_${p}_$pass -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/kernel_lab.py ${PROG[$p]} > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_${p}_$pass.log 2>&1 || { echo "pass $p/$pass failed"; tail -3 $GRAFT_REPO_ROOT/gpurun_out/${TAG}_${p}_$pass.log; exit 1; }
    cd $GRAFT_REPO_ROOT
    echo "pass $p/$pass ok"
  done
done
