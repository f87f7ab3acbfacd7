set -e
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_icp_gpu.py::test_gangs_are_bit_identical > gpurun_out/r06_tests_c.txt 2>&1
SHARD_MODE=contiguous SHARD_N=2,4 timeout -k 10 300 python -u tools/shard_sweep.py auto 64,24,4,0,1,-1,1,8193,-1,96,30,3,16,4 64,24,4,0,1,-1,1,8193,-1,96,30,3,24,4 64,24,4,0,1,-1,1,8193,-1,96,30,3,48,4 64,24,4,0,1,-1,1,8193,-1,96,30,3,48,2 > gpurun_out/r06_mix_sweep2.txt 2>&1
timeout -k 10 300 python -u tools/loky_fanout.py 1 4 8 12 > gpurun_out/r06_loky_fanout.txt 2>&1
for env in "SHARD_SEED=7" "SHARD_SEED=2025 SHARD_DROPOUT=0.35" "SHARD_SEED=11 SHARD_DROPOUT=0.35"; do
  echo "== $env" >> gpurun_out/r06_profile_validation.txt
  env $env SHARD_MODE=contiguous timeout -k 10 300 python -u tools/shard_sweep.py auto 0,0,4,0,2,-1,1,0,-1,16,30,0 0,0,4,0,2,-1,1,0,-1,32,30,0 64,24,4,0,1,-1,1,8193,-1,48,30,3 64,24,4,0,1,-1,1,8193,-1,128,30,3 >> gpurun_out/r06_profile_validation.txt 2>&1
done
