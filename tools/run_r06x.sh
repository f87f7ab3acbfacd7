set -e
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_icp_gpu.py -k "drain or c3_full_stream or gangs_are_bit or timeouts_are" > gpurun_out/r06_tests_x.txt 2>&1
for d in 0 24 12 28 0 24 16; do echo "== drain $d" >> gpurun_out/r06_drain_sweep2.txt; SHARD_DRAIN=$d SHARD_MODE=balanced timeout -k 10 300 python -u tools/shard_sweep.py auto 2>&1 | grep -v amdgpu >> gpurun_out/r06_drain_sweep2.txt; done
