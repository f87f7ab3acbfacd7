set -e
export TMPDIR=/tmp
AB_SHARD=2:0 timeout -k 10 300 python -u tools/ab_probe.py 3 2 4 2>&1 | grep -v amdgpu > gpurun_out/r06_ab_probe2.txt
AB_SHARD=2:1 timeout -k 10 300 python -u tools/ab_probe.py 3 2 4 2>&1 | grep -v amdgpu >> gpurun_out/r06_ab_probe2.txt
AB_SHARD=4:0 timeout -k 10 300 python -u tools/ab_probe.py 4 3 2 2>&1 | grep -v amdgpu >> gpurun_out/r06_ab_probe2.txt
AB_SHARD=8:0 timeout -k 10 300 python -u tools/ab_probe.py 3 2 4 2>&1 | grep -v amdgpu >> gpurun_out/r06_ab_probe2.txt
