set -e
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_icp_gpu.py -k "drain or c3_full_stream or gangs_are_bit or timeouts_are or occupied or mid_batch" > gpurun_out/r06_tests_al.txt 2>&1
timeout -k 10 300 python -u tools/occupy_probe.py 32 64 72 136 2>&1 | grep -v amdgpu > gpurun_out/r06_occupy_probe4.txt
SHARD_TIMING=b2b SHARD_MODE=balanced timeout -k 10 300 python -u tools/shard_sweep.py auto 2>&1 | grep -v amdgpu > gpurun_out/r06_shard_sweep_al.txt
