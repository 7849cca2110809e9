set -u
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_multi.py -x -q -m gpu --timeout 200 --timeout-method thread -k "dropin" > gpurun_out/dropin.log 2>&1; echo "dropin rc=$?"; tail -3 gpurun_out/dropin.log
STEPS=8 DEPTHS=1,3 timeout -k 10 300 python scripts/pipe_time.py ff 1 8 > gpurun_out/pipe_ff_r03.txt 2>&1; echo "pipe rc=$?"; cat gpurun_out/pipe_ff_r03.txt
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tl8 -o run --output-format csv -- python3 scripts/pipe_time.py ff 8 > gpurun_out/tl8.log 2>&1; echo "tl8 rc=$?"
