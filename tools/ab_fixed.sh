#!/bin/bash
# tools/ab_fixed.sh v1 v2 ... : fixed-work timing, interleaved over 3 rounds
for r in 1 2 3; do
  for v in cur "$@"; do
    if [ "$v" = cur ]; then unset SLAMHIP_LIB; else export SLAMHIP_LIB=ab/$v/libslamhip.so; fi
    timeout -k 10 120 python tools/ab_fixed.py 10000 16 5 2>/dev/null || { echo "$v FAILED"; exit 1; }
  done
done
