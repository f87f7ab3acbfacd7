#!/bin/bash
# Strong-scaling shards (rank 0's shard at 2/4/8 ranks) for the current build vs
# ab/ variants, default scheduler: tools/ab_shards.sh v1 v2 ...
for r in 1 2; do
for v in cur "$@"; do
  if [ "$v" = cur ]; then unset SLAMHIP_LIB; else export SLAMHIP_LIB=ab/$v/libslamhip.so; fi
  for n in 5000 2500 1250; do
    res=$(timeout -k 10 120 python bench.py --no-cpu-baseline --no-pgo --steps 10 --pairs $n 2>/dev/null) || { echo "$v $n FAILED"; exit 1; }
    echo "$v pairs $n $(echo "$res" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"], d["parity"]["ok"])')"
  done
done
done | sort
