mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_radix_gpu.py > gpurun_out/pytest_radix.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_radix.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "small or curve or speculation" > gpurun_out/pytest_small.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_small.log
timeout -k 10 120 python tools/mc_small_probe.py > gpurun_out/small_sweep.json 2> gpurun_out/small_sweep.err
TMX_CURVE_SMALL_OFF=1 timeout -k 10 120 python tools/mc_small_probe.py > gpurun_out/small_sweep_off.json 2> gpurun_out/small_sweep_off.err
timeout -k 10 200 python tools/radix_curve_bench.py --mc-steps 20 > gpurun_out/radix_bench.json 2> gpurun_out/radix_bench.err
