set -e
export TMPDIR=/tmp
for env in "SHARD_SEED=2025" "SHARD_SEED=7" "SHARD_SEED=2025 SHARD_DROPOUT=0.35" "SHARD_SEED=11 SHARD_DROPOUT=0.35"; do
  echo "== $env" >> gpurun_out/r06_profile_validation_b2b.txt
  env $env SHARD_TIMING=b2b SHARD_MODE=balanced timeout -k 10 300 python -u tools/shard_sweep.py auto 2>&1 | grep -v amdgpu >> gpurun_out/r06_profile_validation_b2b.txt
done
