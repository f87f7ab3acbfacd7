set -e
export TMPDIR=/tmp
for r in 1 2 3; do
SHARD_N=1 SHARD_MODE=balanced SHARD_WIDE_GROUPS=2 timeout -k 10 300 python -u tools/shard_sweep.py auto auto:2 2,0,4,2,1,-1,1,10001 2,0,4,2,1,2,1,10001 4,0,4,4,1,2,1,10001 2>&1 | grep -v amdgpu >> gpurun_out/r06_wide10k_sweep2.txt
done
for r in 1 2; do
SHARD_N=2,4 SHARD_MODE=balanced timeout -k 10 300 python -u tools/shard_sweep.py auto auto:4 auto:2 2>&1 | grep -v amdgpu >> gpurun_out/r06_probe_sweep2.txt
done
SHARD_SEED=7 SHARD_N=1 SHARD_MODE=balanced SHARD_WIDE_GROUPS=2 timeout -k 10 300 python -u tools/shard_sweep.py auto auto:2 2,0,4,2,1,-1,1,10001 2,0,4,2,1,2,1,10001 2>&1 | grep -v amdgpu >> gpurun_out/r06_wide10k_sweep2.txt
