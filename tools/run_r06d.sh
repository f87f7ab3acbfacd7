set -e
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 380 --timeout-method thread tests/test_icp_gpu.py::test_gangs_are_bit_identical tests/test_icp_gpu.py::test_gang_timeouts_are_repaired > gpurun_out/r06_tests_d.txt 2>&1
for seed in 2025 7; do
  for g in 1 2; do
    echo "== seed $seed wide groups $g" >> gpurun_out/r06_wide_sweep1.txt
    SHARD_SEED=$seed SHARD_WIDE_GROUPS=$g SHARD_N=8 timeout -k 10 300 python -u tools/shard_sweep.py auto 0,0,4,0,2,-1,1,0,-1,32,30,0 0,0,4,0,2,-1,1,0,-1,40,30,0 >> gpurun_out/r06_wide_sweep1.txt 2>&1
  done
done
