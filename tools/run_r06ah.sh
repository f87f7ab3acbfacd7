set -e
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r06_gpu_tests_final.txt 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_smoke_final.txt 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/r06_bench_e.json 2> gpurun_out/r06_bench_e.err
timeout -k 10 600 python -u tools/full_parity.py 10000 16 > gpurun_out/r06_full_parity.json 2> gpurun_out/r06_full_parity.err
bash tools/gpu_profile.sh r06e > gpurun_out/r06e_gpu_profile.log 2>&1
for env in "SHARD_SEED=2025" "SHARD_SEED=7" "SHARD_SEED=2025 SHARD_DROPOUT=0.35" "SHARD_SEED=11 SHARD_DROPOUT=0.35"; do
  echo "== $env" >> gpurun_out/r06_profile_validation6.txt
  env $env timeout -k 10 300 python -u tools/shard_sweep.py auto 2>&1 | grep -v amdgpu >> gpurun_out/r06_profile_validation6.txt
done
