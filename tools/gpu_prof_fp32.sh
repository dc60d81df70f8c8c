cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_curve_anchor_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_anchor.log 2>&1 && tail -2 gpurun_out/pytest_anchor.log && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fp32 -o run --output-format csv -- python3 tools/fp32_curve_bench.py fp32 > gpurun_out/prof_fp32.log 2>&1 && tail -1 gpurun_out/prof_fp32.log && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_UNALIGNED_STALL -d gpurun_out/pmc_fp32 -o pmc --output-format csv -- python3 tools/fp32_curve_bench.py fp32 > gpurun_out/pmc_fp32.log 2>&1 && \
timeout -k 10 300 python tools/fp32_curve_bench.py > gpurun_out/fp32_bench.log 2>&1; cat gpurun_out/fp32_bench.log
