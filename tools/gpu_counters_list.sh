#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
cd /tmp && timeout -k 10 60 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/counters_list.txt 2>&1; echo "list rc $?"
