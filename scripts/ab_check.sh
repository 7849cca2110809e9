set -e
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
tail -1 gpurun_out/pytest_gpu.log
bash scripts/ab.sh "X=0" "VPT_LIB=build_variants/libvpt_prev.so" "X=1"
PMC_PASSES="WRITE_SIZE;FETCH_SIZE" bash scripts/pmc.sh cm
