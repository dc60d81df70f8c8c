# class-count sweep with and without the update lanes (TMX_CURVE_LANES), plus kernel statistics of the lanes run
set -u
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r7f}; mkdir -p $O; export TMPDIR=/tmp
export PROBE_CONFIGS=${PROBE_CONFIGS:-10:1048576,64:1048576,100:262144,256:262144,1000:65536}
timeout -k 10 240 python tools/mc_small_probe.py > $O/lanes_on.log 2>&1 || exit $?
tail -n 1 $O/lanes_on.log
TMX_CURVE_LANES=0 timeout -k 10 240 python tools/mc_small_probe.py > $O/lanes_off.log 2>&1 || exit $?
tail -n 1 $O/lanes_off.log
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o p --output-format csv -- python3 tools/mc_small_probe.py > $O/prof.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_curve_lanes_gpu.py -x -q --timeout 120 --timeout-method thread > $O/lanes_tests.log 2>&1; tail -n 2 $O/lanes_tests.log
