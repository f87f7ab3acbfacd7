set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
SLAMHIP_LIB=ab/t4/libslamhip.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_icp_gpu.py > gpurun_out/t_icp.txt 2>&1
for v in xt4 xt8; do echo "== $v"; SLAMHIP_LIB=ab/$v/libslamhip.so timeout -k 10 150 python tools/lone_pair.py 1118 7264 0 --stamps-all --waves=1024x2 ; done > gpurun_out/lone.txt 2>&1
timeout -k 10 500 tools/ab_run.sh head t2 t4 t8 > gpurun_out/ab1.txt 2>&1
