#!/bin/bash
# Round-6 GPU session steps (one MI355X).  Each step has its own time limit; a step that times out, aborts or
# faults (exit 124 / 134 / 137 / 139) ends the script, any other failure is recorded and the next step runs.
#   usage (from the container): gpurun --timeout 1100 -- bash tools/gpu_r6.sh <out-subdir> step [step ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r6}; shift; mkdir -p "$OUT"; export TMPDIR=/tmp
run() {  # run <name> <seconds> <cmd...>; stdout+stderr -> $OUT/<name>.log
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "step $name rc=$rc"
  case $rc in 124|134|137|139) echo "fatal rc=$rc in $name: stopping"; exit $rc ;; esac
  return 0
}
for s in "$@"; do
  case $s in
    tests) run tests 400 python -u -m pytest ${TMX_TESTS:-tests/test_curve_refit_gpu.py} -m gpu -x -q --timeout 120 --timeout-method thread; tail -3 "$OUT/tests.log" ;;
    kexp) run kexp 120 ./build/kexp_r6/${TMX_KEXP:-exp} ${TMX_KEXP_ARGS:-}; cat "$OUT/kexp.log" ;;
    synclat) for b in 200 1000 1500 3000; do run synclat_$b 120 ./build/kexp_r6/sync_latency_exp 50 $b; cat "$OUT/synclat_$b.log"; done ;;
    kexpmulti) for k in ${TMX_KEXP}; do run kexp_$k 120 ./build/kexp_r6/$k; echo "$k: $(tail -c 400 $OUT/kexp_$k.log)"; done ;;
    kexppmc) run kexppmc 120 rocprofv3 --kernel-trace --pmc ${TMX_PMC:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU} -d "$OUT/kexppmc" -o pmc --output-format csv -- ./build/kexp_r6/${TMX_KEXP:-exp} ;;
    kexppmcmulti) for k in ${TMX_KEXP}; do run kexppmc_$k 120 rocprofv3 --kernel-trace --pmc ${TMX_PMC:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU} -d "$OUT/kexppmc_$k" -o pmc --output-format csv -- ./build/kexp_r6/$k; done ;;
    host) run host 120 python tools/host_overhead_probe.py ;;
    fidprof) run fidprof 200 rocprofv3 --kernel-trace --stats -d "$OUT/fidprof" -o fid --output-format csv -- python3 tools/fid_gram_bench.py ;;
    mifid) run mifid_bench 200 python tools/mifid_bench.py; tail -1 "$OUT/mifid_bench.log" ;;
    kid) run kid_bench 200 python tools/kid_bench.py; tail -1 "$OUT/kid_bench.log" ;;
    fidg) run fid_gram_bench 200 python tools/fid_gram_bench.py; tail -1 "$OUT/fid_gram_bench.log" ;;
    pw) run pairwise_bench 300 python tools/pairwise_bench.py; tail -1 "$OUT/pairwise_bench.log" ;;
    pwprof) run pwprof 300 rocprofv3 --kernel-trace --stats -d "$OUT/pwprof" -o pw --output-format csv -- python3 tools/pairwise_bench.py ;;
    sort) run sort 180 python tools/sort_bench.py; tail -1 "$OUT/sort.log" ;;
    sortsweep) SORT_BENCH_SWEEP=1 run sortsweep 300 python tools/sort_bench.py; tail -1 "$OUT/sortsweep.log" ;;
    sortprof) run sortprof 300 rocprofv3 --kernel-trace --stats -d "$OUT/sortprof" -o sort --output-format csv -- python3 tools/sort_bench.py ;;
    suite) run pytest_gpu 800 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread; tail -3 "$OUT/pytest_gpu.log" ;;
    smoke) run smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"; tail -1 "$OUT/smoke.log" ;;
    fwd) run forward_bench 120 python tools/forward_bench.py; tail -1 "$OUT/forward_bench.log" ;;
    window) run window 120 python tools/window_probe.py ;;
    wsplit) run wsplit 180 python tools/window_split_probe.py; cat "$OUT/wsplit.log" ;;
    fwprof) run fwprof 200 rocprofv3 --kernel-trace -d "$OUT/fwprof" -o fw --output-format csv -- python3 tools/first_window_probe.py base; tail -1 "$OUT/fwprof.log" ;;
    firstwin) for r in 1 2 3; do for v in ${TMX_FW_VARIANTS:-base spin double inplace}; do run fw_${v}_$r 60 python tools/first_window_probe.py $v; tail -1 "$OUT/fw_${v}_$r.log"; done; done ;;
    bench) for i in 1 2; do run bench20_$i 120 python bench.py --steps 20 --warmup 5; tail -1 "$OUT/bench20_$i.log"; done ;;
    bench50) run bench50 120 python bench.py --steps 50 --warmup 5; tail -1 "$OUT/bench50.log" ;;
    prof) run prof 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o headline --output-format csv -- python3 bench.py --steps 20 --warmup 5 ;;
    radix) run radix 300 python tools/radix_curve_bench.py; tail -1 "$OUT/radix.log" ;;
    smallprobe) run smallprobe 240 python tools/mc_small_probe.py; tail -1 "$OUT/smallprobe.log" ;;
    smallab) export PROBE_CONFIGS=${PROBE_CONFIGS:-64:1048576,100:262144,104:262144,256:262144,1000:65536,1001:65536}
             run smallab_on 240 python tools/mc_small_probe.py; tail -1 "$OUT/smallab_on.log"
             TMX_CURVE_SMALL_OFF=1 run smallab_off 240 python tools/mc_small_probe.py; tail -1 "$OUT/smallab_off.log"
             run smallab_prof_on 300 rocprofv3 --kernel-trace --stats -d "$OUT/smallab_prof_on" -o on --output-format csv -- python3 tools/mc_small_probe.py
             TMX_CURVE_SMALL_OFF=1 run smallab_prof_off 300 rocprofv3 --kernel-trace --stats -d "$OUT/smallab_prof_off" -o off --output-format csv -- python3 tools/mc_small_probe.py ;;
    abprobe) export PROBE_CONFIGS=${PROBE_CONFIGS:-64:1048576,100:262144,104:262144,256:262144,10:1048576}
             for v in default ${TMX_AB_VARIANTS:-}; do
               if [ $v = default ]; then unset TMX_NATIVE_LIB; else export TMX_NATIVE_LIB=$PWD/build/ab/$v/_tmx_native.so; fi
               run abprobe_$v 240 python tools/mc_small_probe.py; echo "$v: $(tail -1 $OUT/abprobe_$v.log)"; done; unset TMX_NATIVE_LIB ;;
    abprof) export PROBE_CONFIGS=${PROBE_CONFIGS:-64:1048576,100:262144,104:262144,256:262144,10:1048576,1000:65536,1001:65536}
            run abprof 300 rocprofv3 --kernel-trace --stats -d "$OUT/abprof" -o ab --output-format csv -- python3 tools/mc_small_probe.py ;;
    abpmc) run abpmc 200 rocprofv3 --kernel-trace --pmc ${TMX_PMC:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU} -d "$OUT/abpmc" -o pmc --output-format csv -- python3 tools/mc_small_probe.py ;;
    smallprof) PROBE_SMALL_ONLY=1 run smallprof 300 rocprofv3 --kernel-trace --stats -d "$OUT/smallprof" -o small --output-format csv -- python3 tools/mc_small_probe.py ;;
    radixab) for r in 1 2; do
               TMX_NATIVE_LIB=$PWD/build/ab_radix/_tmx_native.so run radix_old_$r 300 python tools/radix_curve_bench.py; tail -1 "$OUT/radix_old_$r.log"
               run radix_new_$r 300 python tools/radix_curve_bench.py; tail -1 "$OUT/radix_new_$r.log"; done ;;
    radixtest) run radixtest 300 python -u -m pytest tests/test_ops_radix_gpu.py tests/test_binary_samples_gpu.py -x -q --timeout 120 --timeout-method thread; tail -2 "$OUT/radixtest.log" ;;
    radixprof) run radixprof 300 rocprofv3 --kernel-trace --stats -d "$OUT/radixprof" -o radix --output-format csv -- python3 tools/radix_curve_bench.py ;;
    imgprof) run imgprof 900 rocprofv3 --kernel-trace --stats -d "$OUT/imgprof" -o image --output-format csv -- python3 bench.py --config image --steps 1 --warmup 1; tail -2 "$OUT/imgprof.log" ;;
    bertprof) run bertprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/bertprof" -o bert --output-format csv -- python3 bench.py --config bert --steps 2 --warmup 1; tail -2 "$OUT/bertprof.log" ;;
    mapcprof) run mapcprof 300 python tools/map_profile.py; head -c 600 "$OUT/mapcprof.log" ;;
    mapbench) run mapbench 600 python bench.py --config map --steps 5 --warmup 1; tail -1 "$OUT/mapbench.log" ;;
    mapprof) run mapprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/mapprof" -o map --output-format csv -- python3 bench.py --config map --steps 5 --warmup 1; tail -1 "$OUT/mapprof.log" ;;
    sweep) run sweep 300 python tools/class_count_sweep.py; tail -3 "$OUT/sweep.log" ;;
    pmc) run pmc 200 rocprofv3 --kernel-trace --pmc ${TMX_PMC:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU} -d "$OUT/pmc" -o pmc --output-format csv -- python3 bench.py --steps 5 --warmup 2; tail -1 "$OUT/pmc.log" ;;
    wtrace) run wtrace 200 python tools/window_trace.py; tail -c 3000 "$OUT/wtrace.log" ;;
    fwdbench) run fwdbench 200 python tools/forward_bench.py; tail -c 1500 "$OUT/fwdbench.log" ;;
    ccprobe) for v in base spin; do run ccprobe_$v 200 python tools/compute_cost_probe.py $v; tail -c 700 "$OUT/ccprobe_$v.log"; echo; done ;;
    pwx3) PW_SHAPES=${PW_SHAPES:-4096:4096:512,2048:2048:2048,8192:8192:256,10000:10000:2048,16384:2048:1024} PW_DTYPES=float32 PW_MODES=linear,cosine run pwx3 300 python tools/pairwise_bench.py; tail -1 "$OUT/pwx3.log" ;;
    sortitems) for it in 4 8 16; do TMX_OS_ITEMS=$it SORT_BENCH_SWEEP=1 run sortsweep_items$it 300 python tools/sort_bench.py; tail -c 600 "$OUT/sortsweep_items$it.log"; echo; done ;;
    ssimstrip) for st in 256 512 1024; do TMX_SSIM_STRIP=$st run ssim_strip$st 120 ./build/kexp_r6/ssim_mfma_exp; echo "strip $st: $(grep -o '"config4_KS11[^}]*}' $OUT/ssim_strip$st.log | grep -o '"mfma_ms[^,]*')"; done ;;
    ssimbench) run ssimbench 300 python tools/ssim_bench.py; tail -1 "$OUT/ssimbench.log" ;;
    ssimprof) run ssimprof 300 rocprofv3 --kernel-trace --stats -d "$OUT/ssimprof" -o ssim --output-format csv -- python3 tools/ssim_bench.py ;;
    overlap) run overlap 120 python tools/overlap_probe.py; tail -1 "$OUT/overlap.log" ;;
    fwdcprof) run fwdcprof 200 python tools/forward_cprof.py; head -c 4000 "$OUT/fwdcprof.log" ;;
    reduce) run reduce 200 python tools/reduce_bench.py; tail -1 "$OUT/reduce.log" ;;
    *) echo "unknown step $s" ;;
  esac
done
echo "session done"
