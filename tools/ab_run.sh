#!/bin/bash
# C3 bench (ICP only), current build vs ab/ variants, interleaved over 3 rounds
# so box-to-box clock differences cancel.  usage: tools/ab_run.sh v1 v2[@instance] ...
for r in 1 2 3; do
for spec in cur "$@"; do
  # spec: variant[@instance][:probe]
  probe=-1; case "$spec" in *:*) probe=${spec#*:}; spec=${spec%:*};; esac
  v=${spec%@*}; inst=-1; [ "$v" != "$spec" ] && inst=${spec#*@}
  if [ "$v" = cur ]; then unset SLAMHIP_LIB; else export SLAMHIP_LIB=ab/$v/libslamhip.so; fi
  res=$(timeout -k 10 120 python bench.py --no-cpu-baseline --no-pgo --steps 10 --instance $inst --sched-probe $probe 2>/dev/null) || { echo "$spec FAILED"; exit 1; }
  echo "$spec:$probe $(echo "$res" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"], d["roofline"]["pruning_factor"])')"
done
done | sort
