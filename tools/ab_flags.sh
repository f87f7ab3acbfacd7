#!/bin/bash
# C3 bench (ICP only) under different bench.py scheduler flags, interleaved over
# 3 rounds: tools/ab_flags.sh "--sched-warm 0" "--sched-warm 1" ...
for r in 1 2 3; do
for f in "$@"; do
  res=$(timeout -k 10 120 python bench.py --no-cpu-baseline --no-pgo --steps 10 $f 2>/dev/null) || { echo "$f FAILED"; exit 1; }
  echo "[$f] $(echo "$res" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"], d["parity"]["ok"])')"
done
done | sort
