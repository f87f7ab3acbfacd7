set -e
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/occupy_probe.py 72 136 2>&1 | grep -v amdgpu > gpurun_out/r06_occupy_probe3.txt
