set -e
export TMPDIR=/tmp
for seed in 2025 7; do
  echo "== seed $seed wide groups 2" >> gpurun_out/r06_wide_sweep2.txt
  SHARD_SEED=$seed SHARD_WIDE_GROUPS=2 SHARD_N=2,4 timeout -k 10 400 python -u tools/shard_sweep.py auto 0,0,4,0,2,-1,1,8193,-1,48,30,0 0,0,4,0,2,-1,1,8193,-1,64,30,0 64,24,4,0,2,-1,1,8193,-1,48,30,0 64,24,4,0,2,-1,1,8193,-1,64,30,0 0,0,4,0,2,-1,1,8193,-1,96,30,0 >> gpurun_out/r06_wide_sweep2.txt 2>&1
done
