# secondary BASELINE configs on the final tree: BERTScore (config 5), SSIM + PSNR + LPIPS (config 4), mAP (config 3)
set -u
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r7i}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python bench.py --config bert --steps 3 --warmup 1 > $O/bert.log 2>&1 || exit $?
tail -n 1 $O/bert.log | cut -c1-200
timeout -k 10 400 python bench.py --config image --steps 2 --warmup 1 > $O/image.log 2>&1 || exit $?
tail -n 1 $O/image.log | cut -c1-200
timeout -k 10 300 python bench.py --config map --steps 5 --warmup 1 > $O/map.log 2>&1 || exit $?
tail -n 1 $O/map.log | cut -c1-200
