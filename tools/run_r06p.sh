set -e
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_icp_gpu.py::test_gangs_are_bit_identical > gpurun_out/r06_tests_p.txt 2>&1
for seed in 2025 7; do
  echo "== seed $seed" >> gpurun_out/r06_gangk_sweep.txt
  SHARD_SEED=$seed SHARD_MODE=balanced SHARD_N=2 timeout -k 10 400 python -u tools/shard_sweep.py auto 64,24,4,0,1,-1,1,8193,-1,96,30,4 64,24,4,0,1,-1,1,8193,-1,96,30,6 64,24,4,0,1,-1,1,8193,-1,128,30,6 64,24,4,0,1,-1,1,8193,-1,64,30,6 2>&1 | grep -v amdgpu >> gpurun_out/r06_gangk_sweep.txt
done
