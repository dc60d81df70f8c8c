# TMX_SMALL_GRID sweep of the small-class row pass (one process per grid cap): tools/mc_small_probe.py
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/sgrid
export PROBE_CONFIGS=${PROBE_CONFIGS:-10:1048576,100:262144,64:1048576,256:262144}
for rep in 1 2; do
for g in ${SGRID:-0 1024 2048 4096 16384}; do
  TMX_SMALL_GRID=$g timeout -k 10 120 python tools/mc_small_probe.py > gpurun_out/sgrid/g${g}_$rep.log 2>&1 || { echo "fail g=$g rc=$?"; exit 1; }
  echo "grid $g rep $rep: $(tail -1 gpurun_out/sgrid/g${g}_$rep.log)"
done
done
