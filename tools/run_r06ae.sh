set -e
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab_probe.py 3 2 4 2>&1 | grep -v amdgpu > gpurun_out/r06_ab_probe.txt
