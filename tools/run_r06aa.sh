set -e
export TMPDIR=/tmp
for r in 1 2; do
SHARD_N=1 SHARD_MODE=balanced SHARD_WIDE_GROUPS=2 SHARD_DRAIN=0 timeout -k 10 300 python -u tools/shard_sweep.py auto 1,0,4,1,1,-1,1,10001 2,0,4,2,1,-1,1,10001 4,0,4,4,1,-1,1,10001 8,0,4,8,1,-1,1,10001 2>&1 | grep -v amdgpu >> gpurun_out/r06_wide10k_sweep.txt
done
