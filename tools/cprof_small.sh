set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out/cprof
for cn in 10:1048576 64:1048576 256:262144 100:262144; do
  tag=${cn%%:*}
  PROBE_CONFIGS=$cn timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/cprof/c$tag -o c$tag --output-format csv -- python3 tools/mc_small_probe.py > gpurun_out/cprof/c$tag.log 2>&1 || { echo "fail $cn rc=$?"; exit 1; }
  echo "$cn done: $(tail -1 gpurun_out/cprof/c$tag.log | cut -c1-200)"
done
