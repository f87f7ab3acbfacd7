#!/bin/bash
# Strong-scaling projection on ONE GPU: rank 0's shard of the 10k C3 stream at
# 1/2/4/8 ranks (bench.py --pairs P runs the first P pairs), with and without the
# scheduler's CU-exclusive head pairs.  Prints pairs, heads, pairs/s, ms per batch.
for h in 0 64; do
  for n in 10000 5000 2500 1250; do
    r=$(timeout -k 10 120 python bench.py --no-cpu-baseline --no-pgo --steps 10 --pairs $n --sched-heads $h 2>/dev/null) || { echo "$n $h FAILED"; exit 1; }
    echo "pairs $n heads $h $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"])')"
  done
done
