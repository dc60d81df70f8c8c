# round-7 session mAP checks: detection GPU tests, host profile, kernel statistics, bench (each step time-limited)
set -u
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r7b}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ops_detection_gpu.py -x -q --timeout 120 --timeout-method thread > $O/det.log 2>&1; rc=$?; tail -3 $O/det.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/map_profile.py > $O/mapcprof.log 2>&1 || exit $?
head -c 400 $O/mapcprof.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/mapprof -o map --output-format csv -- python3 tools/map_profile.py > $O/mapprof.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config map --steps 5 --warmup 1 > $O/mapbench.log 2>&1 || exit $?
tail -n 1 $O/mapbench.log
