set -e
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gn.py > gpurun_out/r06_gn_tests_j.txt 2>&1
for r in 1 2; do
  for m in 0 32 64 128 200; do
    SLAMHIP_GN_SPLIT_MIN=$m timeout -k 10 120 python -u tools/gn_time.py 2>&1 | grep -v amdgpu | sed "s/^/split_min $m: /" >> gpurun_out/r06_gn_ab_split.txt
  done
done
