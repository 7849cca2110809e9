set -e
mkdir -p gpurun_out
for n in 1 8; do
timeout -k 10 200 python -u scripts/pool_timeline.py ff $n > gpurun_out/tl_$n.log 2>&1
grep -v amdgpu.ids gpurun_out/tl_$n.log
done
