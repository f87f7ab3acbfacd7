set -e
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_icp_gpu.py::test_gangs_are_bit_identical tests/test_icp_gpu.py::test_gang_timeouts_are_repaired > gpurun_out/r06_tests_k.txt 2>&1
timeout -k 10 200 python -u tools/team_stamps.py --wide2 1118 > gpurun_out/r06_wide_stamps5.txt 2>&1
for r in 1 2; do
  for v in cur u2; do
    if [ $v = cur ]; then unset SLAMHIP_LIB; else export SLAMHIP_LIB=ab/$v/libslamhip.so; fi
    for seed in 2025 7; do
      echo "== $v round $r seed $seed" >> gpurun_out/r06_ab_uwin.txt
      SHARD_SEED=$seed SHARD_MODE=balanced SHARD_N=4,8 timeout -k 10 300 python -u tools/shard_sweep.py auto 2>&1 | grep -v amdgpu >> gpurun_out/r06_ab_uwin.txt
    done
  done
done
