set -e
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_icp_gpu.py::test_gangs_are_bit_identical > gpurun_out/r06_tests_b.txt 2>&1
for r in 1 2; do
  for v in cur base; do
    if [ $v = base ]; then export SLAMHIP_LIB=ab/r06base/libslamhip.so; else unset SLAMHIP_LIB; fi
    echo "== $v round $r" >> gpurun_out/r06_ab_widepr.txt
    SHARD_MODE=contiguous SHARD_N=8 timeout -k 10 200 python -u tools/shard_sweep.py auto >> gpurun_out/r06_ab_widepr.txt 2>&1
  done
done
unset SLAMHIP_LIB
SHARD_MODE=contiguous SHARD_N=2,4 timeout -k 10 400 python -u tools/shard_sweep.py 64,24,4,0,1,-1,1,8193,-1,96,30,3,0,2 64,24,4,0,1,-1,1,8193,-1,96,30,3,8,2 64,24,4,0,1,-1,1,8193,-1,96,30,3,16,2 64,24,4,0,1,-1,1,8193,-1,96,30,3,8,4 64,24,4,0,1,-1,1,8193,-1,96,30,3,16,4 64,24,4,0,1,-1,1,8193,-1,96,30,3,32,4 > gpurun_out/r06_mix_sweep1.txt 2>&1
