#!/bin/bash
# default pipelined step with the engine's inter-stream events fenced at system scope (1) or not (0)
export TMPDIR=/tmp
for i in 1 2; do
  for f in 0 1; do
    echo "fence $f: $(SDRG_EVENT_FENCE=$f timeout -k 10 200 python tools/lab/prof_ab.py 2>/dev/null | tail -1)"
  done
done
