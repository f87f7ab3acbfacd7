set -e
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_icp_gpu.py -k "drain or c3_full_stream or gangs_are_bit or timeouts_are or occupied or mid_batch" > gpurun_out/r06_tests_w.txt 2>&1
for d in 0 -1 0 -1; do echo "== drain $d" >> gpurun_out/r06_drain_sweep1.txt; SHARD_DRAIN=$d SHARD_MODE=balanced timeout -k 10 300 python -u tools/shard_sweep.py auto 2>&1 | grep -v amdgpu >> gpurun_out/r06_drain_sweep1.txt; done
