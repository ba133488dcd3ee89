#!/bin/bash
# PMC counters for one configuration (separate passes; kernel-trace only, never sys/runtime traces)
export TMPDIR=/tmp
STAGES=${1:-ssb}
TAG=${2:-pmc}
# (the library is built in-tree on the CPU side before the call)
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d gpurun_out/${TAG}_a -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --stages $STAGES > gpurun_out/${TAG}_a.log 2>&1 || { echo "pmc a failed"; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_IDX_ACTIVE -d gpurun_out/${TAG}_b -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --stages $STAGES > gpurun_out/${TAG}_b.log 2>&1 || { echo "pmc b failed"; exit 1; }
echo pmc done
