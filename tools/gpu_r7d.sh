# per-image COCO route probe: op time with parts of the kernel skipped, plus kernel statistics
set -u
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r7d}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 200 python -u tools/coco_img_probe.py > $O/probe.log 2>&1 || exit $?
tail -n 1 $O/probe.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o p --output-format csv -- python3 tools/coco_img_probe.py > $O/prof.log 2>&1 || exit $?
