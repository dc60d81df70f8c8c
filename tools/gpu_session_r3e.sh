mkdir -p gpurun_out/prof_image
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_ops_image_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3e_tests.log 2>&1 || exit 2
timeout -k 10 400 python bench.py --config image --steps 3 --warmup 1 > gpurun_out/image_cfg.json 2> gpurun_out/image_cfg.err || exit 3
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_image -o image -- python3 bench.py --config image --steps 2 --warmup 1 > gpurun_out/prof_image.log 2>&1 || exit 4
