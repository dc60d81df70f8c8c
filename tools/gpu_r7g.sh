# mAP compute host profile (cProfile) on the current tree
set -u
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r7g}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/map_profile.py > $O/mapcprof.log 2>&1 || exit $?
head -c 300 $O/mapcprof.log
