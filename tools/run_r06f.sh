set -e
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_icp_gpu.py tests/test_bench_multirank_gpu.py tests/test_dist_rccl_gpu.py > gpurun_out/r06_tests_f.txt 2>&1
for env in "SHARD_SEED=2025" "SHARD_SEED=7" "SHARD_SEED=2025 SHARD_DROPOUT=0.35" "SHARD_SEED=11 SHARD_DROPOUT=0.35"; do
  echo "== $env" >> gpurun_out/r06_profile_validation2.txt
  env $env timeout -k 10 300 python -u tools/shard_sweep.py auto >> gpurun_out/r06_profile_validation2.txt 2>&1
done
SHARD_WIDE_GROUPS=2 SHARD_N=2 SHARD_MODE=balanced timeout -k 10 300 python -u tools/shard_sweep.py 64,24,4,0,1,-1,1,8193,-1,96,30,3,16,2 64,24,4,0,1,-1,1,8193,-1,96,30,3,24,2 64,24,4,0,1,-1,1,8193,-1,96,30,3,32,2 > gpurun_out/r06_mix_sweep3.txt 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/r06_bench_a.json 2> gpurun_out/r06_bench_a.err
