hipcc --offload-arch=gfx950 -O3 scripts/ubench_f64.hip -o gpurun_out/ub && timeout -k 10 60 ./gpurun_out/ub > gpurun_out/ub.log 2>&1
