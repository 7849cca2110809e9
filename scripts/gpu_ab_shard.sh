#!/usr/bin/env bash
# A/B of libvpt variants on the 1/8 row-band shard of configs[1] (bench.py --gpus 8's rank 0 workload),
# serialized launches: ms per shard.  usage: bash scripts/gpu_ab_shard.sh name...  ("base" = in-tree)
set -u
for v in "$@"; do
    lib=build_variants/libvpt_$v.so
    [ "$v" = base ] && lib=minimal_volumetric_path_tracer_amd/libvpt.so
    echo "== $v"
    VPT_LIB=$lib STEPS=8 DEPTHS=1 timeout -k 10 200 python scripts/pipe_time.py ff 8 2>&1 | grep "ms/step"
done
