mkdir -p gpurun_out
for k in 1 2 4 8; do TMX_CURVE_CHUNKS=$k timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/bench_chunks_$k.json 2> gpurun_out/bench_chunks_$k.err || exit 3; done
timeout -k 10 200 python tools/sync_audit.py > gpurun_out/sync_audit.json 2> gpurun_out/sync_audit.err || exit 4
