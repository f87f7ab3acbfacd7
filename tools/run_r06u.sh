set -e
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/timeline.py b2:0 b2:1 b8:2 2>&1 | grep -v amdgpu > gpurun_out/r06_timeline_a.txt
SHARD_SEED=7 timeout -k 10 300 python -u tools/timeline.py b8:2 b8:3 2>&1 | grep -v amdgpu > gpurun_out/r06_timeline_b.txt
