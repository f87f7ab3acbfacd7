#!/bin/bash
# Strong-scaling projection with gangs (one GPU): rank 0's shard of the 10k C3
# stream at 2/4/8 ranks for several (gangs, parts) settings and head counts.
# Prints pairs, heads, gangs, pairs/s, ms per batch.
set -- ${@:-64 0,2 64 8,4 64 8,5 64 16,4 64 4,4 64 8,3 64 8,6}
while [ $# -ge 2 ]; do
  h=$1; g=$2; shift 2
  for n in 5000 2500 1250; do
    r=$(timeout -k 10 120 python bench.py --no-cpu-baseline --no-pgo --steps 10 --pairs $n --sched-heads $h --sched-gangs $g 2>/dev/null) || { echo "$n $h $g FAILED"; exit 1; }
    echo "pairs $n heads $h gangs $g $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"], d["parity"]["ok"])')"
  done
done
