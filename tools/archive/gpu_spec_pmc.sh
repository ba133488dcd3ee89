#!/bin/bash
# Spectrum kernel counters (one pass per counter group, kernel-trace only): where does a frame's time go?
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/avail.txt 2>&1 || true
grep -oE "^[[:space:]]*(SQ|SQC|TA|TD|TCP)_[A-Z0-9_]+" gpurun_out/avail.txt | sort -u | tr -d ' ' > gpurun_out/avail_sq.txt || true
run() { timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $2 -d gpurun_out/spmc_$1 -o run --output-format csv -- python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --stages spectrum > gpurun_out/spmc_$1.log 2>&1 || { echo "pass $1 failed"; tail -3 gpurun_out/spmc_$1.log; exit 1; }; echo "pass $1 ok"; }
run a "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU"
run b "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
run c "SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_CVT SQ_WAIT_ANY SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_BUSY_CU_CYCLES"
