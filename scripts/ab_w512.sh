# A/B of the 512-thread shared-pool variants (full image via scripts/ab.sh; 1/8 shard via pipe_time)
set -e
B=build_variants
bash scripts/ab.sh "VPT_LIB=$B/libvpt_w512.so" "VPT_LIB=$B/libvpt_w512u.so" "VPT_LIB=$B/libvpt_w512s.so" "VPT_LIB=$B/libvpt_w512p.so" "X=0" "VPT_LIB=$B/libvpt_w512.so"
DEPTHS=1,3 timeout -k 10 200 python -u scripts/pipe_time.py ff 8 2>&1 | grep -v amdgpu
VPT_LIB=$B/libvpt_w512.so DEPTHS=1,3 timeout -k 10 200 python -u scripts/pipe_time.py ff 8 2>&1 | grep -v amdgpu
