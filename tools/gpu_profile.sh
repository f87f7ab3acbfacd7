#!/bin/bash
# Round profiling recipe (run on the GPU box from the repo root):
#   kernel trace + stats of the bench, then FETCH_SIZE and WRITE_SIZE in
#   separate PMC passes (MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE need
#   separate passes; FETCH_SIZE under-reports wide coalesced reads by 2x), then
#   the instruction mix (VALU / SALU / LDS instructions, waves).
set -e
TAG=${1:-r04}
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o icp -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pgo > $OUT/bench_traced.json 2> $OUT/bench_traced.err
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o f -- \
    python3 tools/prof_icp.py 10000 1 > $OUT/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o w -- \
    python3 tools/prof_icp.py 10000 1 > $OUT/pmc_write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES --output-format csv -d $OUT/pmc_inst -o i -- \
    python3 tools/prof_icp.py 10000 1 > $OUT/pmc_inst.log 2>&1
# VALU busy fraction from counters (not an assumed cycles-per-instruction):
# SQ_ACTIVE_INST_VALU (quad-cycles, summed over waves) x 4 over the SIMD-cycles
# of the dispatch (GRBM_GUI_ACTIVE, summed over the 8 XCDs)
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE \
    --output-format csv -d $OUT/pmc_busy -o b -- python3 tools/prof_icp.py 10000 1 > $OUT/pmc_busy.log 2>&1
find $OUT -name "*.csv" | head -20
