mkdir -p gpurun_out/pmc_small2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "small or speculation or curve_hist or rare" > gpurun_out/small_tests.log 2>&1 || exit 2
PROBE_SMALL_ONLY=1 timeout -k 10 120 python tools/mc_small_probe.py > gpurun_out/splits_default.json 2>/dev/null || exit 3
PROBE_SMALL_ONLY=1 timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES --kernel-trace -d gpurun_out/pmc_small2 -o pmc -- python3 tools/mc_small_probe.py > gpurun_out/pmc_small2.log 2>&1 || exit 4
