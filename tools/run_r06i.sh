set -e
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r06_gpu_tests_i.txt 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_smoke_i.txt 2>&1
bash tools/gpu_profile.sh r06a > gpurun_out/r06a_gpu_profile.log 2>&1
mkdir -p gpurun_out/gnprof_r06
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gnprof_r06 -o gn -- python3 tools/prof_gn.py 10 > gpurun_out/gnprof_r06.log 2>&1
