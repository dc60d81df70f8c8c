# LPIPS channels_last trunk: image GPU tests, then BASELINE config 4 with the trunk in NCHW vs channels_last
set -u
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r7l}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_ops_image_gpu.py tests/unittests/image -m gpu -x -q --timeout 120 --timeout-method thread > $O/img_tests.log 2>&1; rc=$?; tail -n 1 $O/img_tests.log; [ $rc -eq 0 ] || exit $rc
TMX_LPIPS_CHANNELS_LAST=1 timeout -k 10 400 python bench.py --config image --steps 2 --warmup 1 > $O/image_cl.log 2>&1 || exit $?
tail -n 1 $O/image_cl.log | cut -c1-160
TMX_LPIPS_CHANNELS_LAST=0 timeout -k 10 400 python bench.py --config image --steps 2 --warmup 1 > $O/image_nchw.log 2>&1 || exit $?
tail -n 1 $O/image_nchw.log | cut -c1-160
