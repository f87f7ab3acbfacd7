set -e
export TMPDIR=/tmp
for r in 1 2; do
  for v in cur pre; do
    if [ $v = cur ]; then unset SLAMHIP_LIB; else export SLAMHIP_LIB=ab/$v/libslamhip.so; fi
    for seed in 2025 7; do
      echo "== $v round $r seed $seed" >> gpurun_out/r06_ab_opaque.txt
      SHARD_SEED=$seed SHARD_MODE=balanced SHARD_N=2 timeout -k 10 300 python -u tools/shard_sweep.py auto 2>&1 | grep -v amdgpu >> gpurun_out/r06_ab_opaque.txt
    done
  done
done
