mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "small or curve or speculation" > gpurun_out/pytest_small.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_small.log
timeout -k 10 120 python tools/mc_small_probe.py > gpurun_out/small_sweep.json 2> gpurun_out/small_sweep.err
TMX_CURVE_SMALL_OFF=1 timeout -k 10 120 python tools/mc_small_probe.py > gpurun_out/small_sweep_off.json 2> gpurun_out/small_sweep_off.err
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_r3a.json 2> gpurun_out/bench_r3a.err
