#!/bin/bash
# Stall breakdown of the batched ICP kernel per variant (GPU box):
#   tools/ab_pmc.sh cur nosticky ...   -> gpurun_out/abpmc/<variant>/...
export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SALU SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE"
for v in "$@"; do
  if [ "$v" = cur ]; then unset SLAMHIP_LIB; else export SLAMHIP_LIB=ab/$v/libslamhip.so; fi
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/abpmc/$v -o p -- \
      python3 tools/prof_icp.py 10000 1 > gpurun_out/abpmc/$v.log 2>&1 || { echo "$v failed"; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/abpmc "$@"
