mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "small or speculation or curve_hist_multiclass" > gpurun_out/small_tests.log 2>&1 || exit 2
PROBE_SMALL_ONLY=1 timeout -k 10 120 python tools/mc_small_probe.py > gpurun_out/splits_default.json 2>/dev/null || exit 3
for sp in 8 16 32 64 128; do TMX_SMALL_SPLITS=$sp PROBE_SMALL_ONLY=1 timeout -k 10 120 python tools/mc_small_probe.py > gpurun_out/splits_$sp.json 2>/dev/null || exit 3; done
