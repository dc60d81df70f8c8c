mkdir -p gpurun_out/prof_image
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
TMX_LPIPS_NCHW=1 timeout -k 10 500 python bench.py --config image --steps 2 --warmup 1 > gpurun_out/image_cfg_nchw.json 2> gpurun_out/image_cfg_nchw.err || exit 3
timeout -k 10 600 python bench.py --config image --steps 2 --warmup 1 > gpurun_out/image_cfg.json 2> gpurun_out/image_cfg.err || exit 4
