set -e
export TMPDIR=/tmp
SHARD_MODE=balanced SHARD_N=2,4 timeout -k 10 500 python -u tools/shard_sweep.py auto auto:2 auto:4 auto:5 auto:6 auto:8 2>&1 | grep -v amdgpu > gpurun_out/r06_probe_sweep.txt
