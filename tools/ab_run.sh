#!/bin/bash
# Run the C3 bench (ICP only) for the current build and each ab/ variant given.
# usage (GPU box): tools/ab_run.sh variant1 variant2[@instance] ...
for spec in cur "$@"; do
  v=${spec%@*}; inst=-1; [ "$v" != "$spec" ] && inst=${spec#*@}
  if [ "$v" = cur ]; then unset SLAMHIP_LIB; else export SLAMHIP_LIB=ab/$v/libslamhip.so; fi
  r=$(timeout -k 10 120 python bench.py --no-cpu-baseline --no-pgo --steps 10 --instance $inst 2>/dev/null) || { echo "$spec FAILED"; exit 1; }
  echo "$spec $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"], d["roofline"]["pruning_factor"])')"
done
