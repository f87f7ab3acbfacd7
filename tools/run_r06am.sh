set -e
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r06_gpu_tests_final2.txt 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_smoke_final2.txt 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/r06_bench_f.json 2> gpurun_out/r06_bench_f.err
timeout -k 10 600 python -u tools/full_parity.py 10000 16 > gpurun_out/r06_full_parity.json 2> gpurun_out/r06_full_parity.err
bash tools/gpu_profile.sh r06f > gpurun_out/r06f_gpu_profile.log 2>&1
timeout -k 10 300 python -u tools/occupy_probe.py 32 72 136 2>&1 | grep -v amdgpu > gpurun_out/r06_occupy_probe5.txt
