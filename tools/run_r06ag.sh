set -e
export TMPDIR=/tmp
for sh in 2:0 4:0 4:2 8:0 8:2; do AB_KNOB=drain AB_SHARD=$sh timeout -k 10 300 python -u tools/ab_probe.py 0 24 2>&1 | grep -v amdgpu >> gpurun_out/r06_ab_drain.txt; done
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_icp_gpu.py -k "drain or c3_full_stream or gangs_are_bit" > gpurun_out/r06_tests_ag.txt 2>&1
