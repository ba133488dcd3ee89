#!/bin/bash
# functional rehearsal of bench.py's N > 1 path on a one-GPU box (gloo, both ranks on cuda:0)
export TMPDIR=/tmp
mkdir -p gpurun_out
for G in records+focus records+pcm+focus; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 \
      bench.py --gpus 2 --steps 5 --warmup 2 --rehearse-gloo --gather $G --streams 1024 > gpurun_out/rehearse_$G.log 2>&1 || { echo "rehearsal $G failed"; tail -30 gpurun_out/rehearse_$G.log; exit 1; }
  grep metric gpurun_out/rehearse_$G.log | python3 -c "
import sys, json; d = json.loads(sys.stdin.read()); print('$G', d['n_gpus'], d['value'], d['config']['parallelism'], d['pipelined'], d.get('rehearsal_check'))"
done
