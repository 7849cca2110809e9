set -e
mkdir -p gpurun_out
for b in 16 8 4; do
ALL_RANKS=1 BAND_ROWS=$b timeout -k 10 200 python -u scripts/shard_time.py ff 1 8 > gpurun_out/shard_b$b.log 2>&1
cat gpurun_out/shard_b$b.log | grep -v amdgpu.ids
done
