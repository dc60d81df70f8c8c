# round-6b checks: detection GPU tests + mAP bench (reverted accumulate grid) + class-count sweep, each step time-limited
set -u
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r7c}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ops_detection_gpu.py -x -q --timeout 120 --timeout-method thread > $O/det.log 2>&1; rc=$?; tail -1 $O/det.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/mapprof -o map --output-format csv -- python3 tools/map_profile.py > $O/mapprof.log 2>&1 || exit $?
for i in 1 2; do timeout -k 10 300 python bench.py --config map --steps 5 --warmup 1 > $O/mapbench_$i.log 2>&1 || exit $?; tail -n 1 $O/mapbench_$i.log; done
timeout -k 10 240 python tools/mc_small_probe.py > $O/smallprobe.log 2>&1 || exit $?
tail -n 1 $O/smallprobe.log
