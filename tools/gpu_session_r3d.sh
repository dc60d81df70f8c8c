mkdir -p gpurun_out/prof_ssim2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_ops_image_gpu.py tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "ssim or fused or small or speculation" > gpurun_out/r3d_tests.log 2>&1 || exit 2
timeout -k 10 200 python tools/ssim_bench.py > gpurun_out/ssim_v2b.json 2> gpurun_out/ssim_v2b.err || exit 4
SSIM_B=32 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ssim2 -o ssim -- python3 tools/ssim_bench.py > gpurun_out/prof_ssim2.log 2>&1 || exit 7
