set -e
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/timeline.py b4:0 b4:3 b2:0 2>&1 | grep -v amdgpu > gpurun_out/r06_timeline_c.txt
