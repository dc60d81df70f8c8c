mkdir -p gpurun_out
for sp in 1 2 4 8 16 32 64; do TMX_SMALL_SPLITS=$sp PROBE_SMALL_ONLY=1 timeout -k 10 120 python tools/mc_small_probe.py > gpurun_out/splits_$sp.json 2>/dev/null || exit 3; done
