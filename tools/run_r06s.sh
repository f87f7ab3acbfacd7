set -e
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/single_phase_probe.py 2025 7 2>&1 | grep -v amdgpu > gpurun_out/r06_single_phase.txt
