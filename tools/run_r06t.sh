set -e
export TMPDIR=/tmp
for s in 7 2025; do timeout -k 10 300 python -u tools/shard_stats.py $s 8 2>&1 | grep -v amdgpu >> gpurun_out/r06_shard_stats.txt; done
