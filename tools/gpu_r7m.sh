# BASELINE config 4 kernel statistics with the LPIPS trunk in channels_last vs NCHW (one short run each)
set -u
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r7m}; mkdir -p $O; export TMPDIR=/tmp
TMX_LPIPS_CHANNELS_LAST=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/cl -o cl --output-format csv -- python3 bench.py --config image --steps 1 --warmup 1 > $O/cl.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/nchw -o nchw --output-format csv -- python3 bench.py --config image --steps 1 --warmup 1 > $O/nchw.log 2>&1 || exit $?
