set -e
export TMPDIR=/tmp
for r in 1 2; do
SHARD_N=1 SHARD_MODE=balanced timeout -k 10 300 python -u tools/shard_sweep.py auto auto:1 auto:2 2>&1 | grep -v amdgpu >> gpurun_out/r06_probe_sweep3.txt
SHARD_N=8 SHARD_MODE=balanced timeout -k 10 300 python -u tools/shard_sweep.py auto auto:2 auto:4 2>&1 | grep -v amdgpu >> gpurun_out/r06_probe_sweep3.txt
done
SHARD_SEED=7 SHARD_N=2,8 SHARD_MODE=balanced timeout -k 10 300 python -u tools/shard_sweep.py auto auto:2 auto:4 2>&1 | grep -v amdgpu >> gpurun_out/r06_probe_sweep3.txt
