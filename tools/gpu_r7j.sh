# LPIPS trunk memory-format probe (NCHW vs channels_last)
set -u
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r7j}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u tools/lpips_layout_probe.py > $O/lpips_layout.log 2>&1 || exit $?
tail -n 3 $O/lpips_layout.log
