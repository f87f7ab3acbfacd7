#!/bin/bash
# Strong-scaling shards (rank 0's shard of the 10k C3 stream at 2/4/8 ranks,
# and the full 10k batch) for scheduler settings given as
# "BULK WIDE GANGS HEADS" quadruples (bench.py --bulk-gangs / --sched-wide /
# --sched-gangs / --sched-heads).  Prints pairs, settings, pairs/s, ms, parity.
set -- ${@:-0,2 0,1 24,4 64  4096,2 0,1 24,4 64  4096,3 0,1 24,4 64  4096,2 1,1 24,4 64  4096,2 0,1 0,4 0}
while [ $# -ge 4 ]; do
  bg=$1; w=$2; g=$3; h=$4; shift 4
  for n in 10000 5000 2500 1250; do
    r=$(timeout -k 10 120 python bench.py --no-cpu-baseline --no-pgo --steps 10 --pairs $n --bulk-gangs $bg --sched-wide $w --sched-gangs $g --sched-heads $h 2>/dev/null) || { echo "$n $bg $w $g $h FAILED"; exit 1; }
    echo "pairs $n bulk $bg wide $w gangs $g heads $h $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"], d["parity"]["ok"])')"
  done
done
