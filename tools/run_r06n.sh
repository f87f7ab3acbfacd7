set -e
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 380 --timeout-method thread tests/test_icp_gpu.py::test_gangs_are_bit_identical tests/test_icp_gpu.py::test_gang_timeouts_are_repaired > gpurun_out/r06_tests_n.txt 2>&1
timeout -k 10 200 python -u tools/team_stamps.py --wide2 1118 > gpurun_out/r06_wide_stamps7.txt 2>&1
for seed in 2025 7; do
  echo "== seed $seed" >> gpurun_out/r06_wide_sweep4.txt
  SHARD_SEED=$seed SHARD_MODE=balanced timeout -k 10 300 python -u tools/shard_sweep.py auto 2>&1 | grep -v amdgpu >> gpurun_out/r06_wide_sweep4.txt
done
for seed in 2025 7; do
  echo "== seed $seed wide groups 1 (explicit, share 2)" >> gpurun_out/r06_wide_sweep4.txt
  SHARD_SEED=$seed SHARD_MODE=balanced SHARD_WIDE_GROUPS=1 SHARD_N=8 timeout -k 10 300 python -u tools/shard_sweep.py 0,0,4,0,2,-1,1,0,-1,40,30,0 2>&1 | grep -v amdgpu >> gpurun_out/r06_wide_sweep4.txt
  SHARD_SEED=$seed SHARD_MODE=balanced SHARD_WIDE_GROUPS=1 SHARD_N=4 timeout -k 10 300 python -u tools/shard_sweep.py 0,0,4,0,2,-1,1,8193,-1,64,30,0 2>&1 | grep -v amdgpu >> gpurun_out/r06_wide_sweep4.txt
done
timeout -k 10 200 python -u tools/team_stamps.py --wide 1118 > gpurun_out/r06_wide_stamps8.txt 2>&1
