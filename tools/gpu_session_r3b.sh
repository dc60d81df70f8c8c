mkdir -p gpurun_out/prof_small gpurun_out/prof_radix
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_ops_detection_gpu.py tests/test_ops_radix_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/det_radix_tests.log 2>&1 || exit 2
timeout -k 10 300 python tools/segm_map_bench.py --check > gpurun_out/segm_bench.json 2> gpurun_out/segm_bench.err || exit 3
PROBE_SMALL_ONLY=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_small -o small -- python3 tools/mc_small_probe.py > gpurun_out/prof_small.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_radix -o radix -- python3 tools/radix_curve_bench.py --mc-steps 4 > gpurun_out/prof_radix.log 2>&1 || exit 5
