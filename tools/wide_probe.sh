#!/bin/bash
# Strong-scaling shards (rank 0's shard of the 10k C3 stream at 2/4/8 ranks)
# with the wide tier: "W,S G,K" settings (wide pairs, LDS share; gangs, parts).
# Prints pairs, wide, gangs, pairs/s, ms per batch, parity.
set -- ${@:-0,1 24,4 2,1 24,4 4,1 24,4 8,1 24,4 4,2 24,4 8,2 24,4}
while [ $# -ge 2 ]; do
  w=$1; g=$2; shift 2
  for n in 5000 2500 1250; do
    r=$(timeout -k 10 120 python bench.py --no-cpu-baseline --no-pgo --steps 10 --pairs $n --sched-wide $w --sched-gangs $g 2>/dev/null) || { echo "$n $w $g FAILED"; exit 1; }
    echo "pairs $n wide $w gangs $g $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"], d["parity"]["ok"])')"
  done
done
