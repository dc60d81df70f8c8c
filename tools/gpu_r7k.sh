# final-tree checks: smoke, full GPU suite, LPIPS trunk layout probe (each step time-limited)
set -u
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r7k}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -n 1 $O/smoke.log
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -n 1 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/lpips_layout_probe.py > $O/lpips_layout.log 2>&1 || exit $?
tail -n 1 $O/lpips_layout.log
