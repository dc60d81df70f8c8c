# mAP: detection tests (both sort keys), op probe stable vs unique sort key, kernel stats, bench
set -u
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r7h}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ops_detection_gpu.py -x -q --timeout 120 --timeout-method thread > $O/det.log 2>&1; rc=$?; tail -1 $O/det.log; [ $rc -eq 0 ] || exit $rc
TMX_COCO_SORT_UNIQUE=1 timeout -k 10 300 python -u -m pytest tests/test_ops_detection_gpu.py -x -q --timeout 120 --timeout-method thread > $O/det_unique.log 2>&1; rc=$?; tail -1 $O/det_unique.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/coco_img_probe.py > $O/probe.log 2>&1 || exit $?
tail -n 1 $O/probe.log
TMX_COCO_SORT_UNIQUE=1 timeout -k 10 200 python -u tools/coco_img_probe.py > $O/probe_unique.log 2>&1 || exit $?
tail -n 1 $O/probe_unique.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o p --output-format csv -- python3 tools/coco_img_probe.py > $O/prof.log 2>&1 || exit $?
for i in 1 2; do timeout -k 10 300 python bench.py --config map --steps 5 --warmup 1 > $O/mapbench_$i.log 2>&1 || exit $?; tail -n 1 $O/mapbench_$i.log | cut -c1-60; done
