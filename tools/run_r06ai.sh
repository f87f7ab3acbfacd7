set -e
export TMPDIR=/tmp
AB_KNOB=wide timeout -k 10 300 python -u tools/ab_probe.py 0 2 4 2>&1 | grep -v amdgpu > gpurun_out/r06_ab_wide10k.txt
