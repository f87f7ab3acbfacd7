set -e
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/occupy_probe.py 16 32 64 2>&1 | grep -v amdgpu > gpurun_out/r06_occupy_probe1.txt
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_icp_gpu.py::test_occupied_cus_do_not_stall_the_exchange_tiers tests/test_icp_gpu.py::test_gang_timeouts_are_repaired tests/test_icp_gpu.py::test_gangs_are_bit_identical > gpurun_out/r06_tests_r.txt 2>&1
SHARD_MODE=balanced timeout -k 10 300 python -u tools/shard_sweep.py auto 2>&1 | grep -v amdgpu > gpurun_out/r06_shard_sweep_r.txt
