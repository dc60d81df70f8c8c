mkdir -p gpurun_out/pmc_small
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/pmc_small/avail.txt 2>&1 || true
timeout -k 10 300 python tools/radix_curve_bench.py --mc-steps 4 > gpurun_out/radix_bench2.json 2> gpurun_out/radix_bench2.err || exit 3
PROBE_SMALL_ONLY=1 timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES --kernel-trace -d gpurun_out/pmc_small -o pmc -- python3 tools/mc_small_probe.py > gpurun_out/pmc_small.log 2>&1 || exit 4
