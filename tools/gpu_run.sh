# One GPU-box session: `bash tools/gpu_run.sh TAG STEP...` runs the named steps
# in order, each under its own time limit, output under gpurun_out/TAG/, and
# stops at the first failing step (no GPU work after a fault or a time-out).
# Steps:
#   bench      python bench.py --gpus 1 --steps 20 --warmup 5 (the driver's exact N=1 command)
#   benchlong  python bench.py (200 steps, 20 warmup)
#   gloo2      bench.py --gpus 2 --dist-backend gloo (two ranks on one GPU)
#   forcedist  bench.py --force-dist (one-rank RCCL: the captured per-step collective)
#   pytest     pytest -m gpu (every GPU test)
#   pytest:F   pytest -m gpu on tests/F only
#   smoke      __graft_entry__.smoke()
#   rocprof    rocprofv3 --kernel-trace --stats of a short bench command
#   abc        tools/ab_chamfer.py (same-box Chamfer variant A/B)
#   abe        tools/ab_emd.py   (same-box EMD variant A/B)
#   grid       GPU tests of the grid forward, tools/grid_diag.py, tools/ab_grid.py
#   gridkt     rocprofv3 --kernel-trace --stats of tools/grid_diag.py
#   pmc        tools/pmc_passes.sh (kernel trace of bench + one counter pass per group)
#   stamps     tools/stamp_filt.py fused 7 11 (needs `make stamps`)
#   stampslg   tools/stamp_lgrid.py 13 and 11 (needs `make stamps`)
#   probe      tools/probe_replay.py (timed-region overhead by launch form)
#   benchab    the driver's bench command twice per side-leg order (same box)
#   probeev    tools/probe_events.py (does recording the region's timing events cost wall time)
#   abcl       tools/ab_chamfer.sh (the A/B across lib/libpcm_hip_{base,v*}.so builds, twice)
#   emddiag    tools/emd_diag.py: config 3 per iteration, the training call by bidder count
#   abr        tools/ab_ref_call.py (the unchanged caller's pieces: forward geometries, strided backward)
#   abf        tools/ab_layout_forms.py (the training call's mixed-layout step: two forwards vs one), twice
#   abl        tools/ab_launch_form.py (N=1 region: direct C loop against the warmed 20-step graph)
#   gfc        tools/grid_first_call.py in fresh processes (+ a per-call kernel trace)
#   gfc2       12 fresh processes under rocprofv3 --kernel-trace, fp32-first and fp16-first orders
#   tct        rocprofv3 kernel traces of tools/training_call_trace.py {after,before,reference}
set -o pipefail
TAG=$1
shift
O=gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
for S in "$@"; do
    echo "[gpu_run] $S $(date +%T)"
    case "$S" in
    bench) timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench.json" 2> "$O/bench.err" ;;
    benchlong) timeout -k 10 600 python -u bench.py > "$O/benchlong.json" 2> "$O/benchlong.err" ;;
    gloo2) timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 --no-cpu \
               --no-emd --no-dense --no-icp --no-ref-call > "$O/gloo2.json" 2> "$O/gloo2.err" ;;
    forcedist) timeout -k 10 300 python -u bench.py --force-dist --steps 50 --warmup 5 --no-cpu --no-emd \
               --no-dense --no-icp --no-ref-call > "$O/forcedist.json" 2> "$O/forcedist.err" ;;
    pytest) timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
               > "$O/pytest.txt" 2>&1 ;;
    pytest:*) timeout -k 10 600 python -u -m pytest "tests/${S#pytest:}" -m gpu -x -q --timeout 120 \
               --timeout-method thread > "$O/pytest_${S#pytest:}.txt" 2>&1 ;;
    smoke) timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' \
               > "$O/smoke.txt" 2>&1 ;;
    rocprof) (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof" \
               -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 --no-cpu > "$GRAFT_REPO_ROOT/$O/rocprof_bench.json" \
               2> "$GRAFT_REPO_ROOT/$O/rocprof.err") ;;
    abc) AB_VARIANTS=${AB_VARIANTS:-11,15} timeout -k 10 600 python -u tools/ab_chamfer.py > "$O/ab_chamfer.txt" 2>&1 &&
         AB_VARIANTS=${AB_VARIANTS:-11,15} timeout -k 10 600 python -u tools/ab_chamfer.py >> "$O/ab_chamfer.txt" 2>&1 ;;
    abcc) AB_COLD=${AB_COLD:-0.3} AB_VARIANTS=${AB_VARIANTS:-11,15} timeout -k 10 600 python -u tools/ab_chamfer.py \
               > "$O/ab_chamfer_cold.txt" 2>&1 &&
          AB_COLD=${AB_COLD:-0.3} AB_VARIANTS=${AB_VARIANTS:-11,15} timeout -k 10 600 python -u tools/ab_chamfer.py \
               >> "$O/ab_chamfer_cold.txt" 2>&1 ;;
    abgl) for r in 1 2 3; do for lib in base default; do
              if [ $lib = base ]; then L=$PWD/3d-pointcloudreconstruction_amd/lib/libpcm_hip_base.so; else L=$PWD/3d-pointcloudreconstruction_amd/lib/libpcm_hip.so; fi
              PCM_HIP_LIB=$L timeout -k 10 120 python -u tools/ab_grid_libs.py >> "$O/ab_grid_libs.txt" 2>&1 || exit 1
          done; done ;;
    abe) timeout -k 10 600 python -u tools/ab_emd.py > "$O/ab_emd.txt" 2>&1 ;;
    grid) timeout -k 10 600 python -u -m pytest tests/test_chamfer_grid_gpu.py -m gpu -x -q --timeout 120 \
               --timeout-method thread > "$O/pytest_grid.txt" 2>&1 &&
          timeout -k 10 300 python -u tools/grid_diag.py > "$O/grid_diag.txt" 2>&1 &&
          timeout -k 10 300 python -u tools/ab_grid.py > "$O/ab_grid.txt" 2>&1 ;;
    gridkt) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/gridkt" -o grid --output-format csv \
               -- python3 tools/grid_diag.py > "$O/gridkt.log" 2>&1 ;;
    pmc) timeout -k 10 900 bash tools/pmc_passes.sh "$O/pmc" > "$O/pmc_passes.log" 2>&1 ;;
    stamps) PCM_HIP_LIB=$PWD/3d-pointcloudreconstruction_amd/lib/libpcm_hip_stamps.so \
            PCM_HIP_TUNE_LIB=$PWD/3d-pointcloudreconstruction_amd/lib/libpcm_hip_stamps.so timeout -k 10 300 \
               python -u tools/stamp_filt.py fused 15 > "$O/stamps_fused.txt" 2>&1 ;;
    stampslg) timeout -k 10 300 python -u tools/stamp_lgrid.py 13 > "$O/stamps_lgrid.txt" 2>&1 &&
              timeout -k 10 300 python -u tools/stamp_lgrid.py 11 >> "$O/stamps_lgrid.txt" 2>&1 ;;
    probe) timeout -k 10 300 python -u tools/probe_replay.py > "$O/probe_replay.txt" 2>&1 &&
           timeout -k 10 300 python -u tools/probe_timed.py > "$O/probe_timed.txt" 2>&1 ;;
    abcl) timeout -k 10 900 bash tools/ab_chamfer.sh > "$O/ab_chamfer_libs.txt" 2>&1 ;;
    emddiag) timeout -k 10 300 python -u tools/emd_diag.py --per-iter > "$O/emd_diag_c3.txt" 2>&1 &&
             timeout -k 10 300 python -u tools/emd_diag.py --train --by-nu > "$O/emd_diag_train.txt" 2>&1 ;;
    emdstamps) PCM_HIP_LIB=$PWD/3d-pointcloudreconstruction_amd/lib/libpcm_hip_stamps.so timeout -k 10 300 \
               python -u tools/emd_diag.py > "$O/emd_stamps_c3.txt" 2>&1 ;;
    abrl) for r in 1 2; do for lib in base default; do
              if [ $lib = base ]; then L=$PWD/3d-pointcloudreconstruction_amd/lib/libpcm_hip_base.so; else L=$PWD/3d-pointcloudreconstruction_amd/lib/libpcm_hip.so; fi
              echo "== $lib" >> "$O/ab_ref_call_libs.txt"
              PCM_HIP_LIB=$L timeout -k 10 300 python -u tools/ab_ref_call.py >> "$O/ab_ref_call_libs.txt" 2>&1 || exit 1
          done; done ;;
    abr) timeout -k 10 300 python -u tools/ab_ref_call.py > "$O/ab_ref_call.txt" 2>&1 ;;
    gfc) for o in f32,f32,f32,f16,f16 f16,f16,f32,f32 dense,tiny,f32,f32 ; do
             timeout -k 10 120 python -u tools/grid_first_call.py $o >> "$O/grid_first_call.txt" 2>&1 || exit 1
         done
         (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/$O/gfc_kt" -o run \
             --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/grid_first_call.py" f32,f32,f32,f16,f16 \
             > "$GRAFT_REPO_ROOT/$O/gfc_kt.log" 2>&1) ;;
    gfc2) for r in 1 2 3 4 5 6; do for o in f32,f32,f16,f16 f16,f16,f32,f32; do
             (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/$O/gfc2/${o}_$r" -o run \
                 --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/grid_first_call.py" $o \
                 > "$GRAFT_REPO_ROOT/$O/gfc2_${o}_$r.log" 2>&1) || exit 1
         done; done ;;
    abf) timeout -k 10 300 python -u tools/ab_layout_forms.py > "$O/ab_layout_forms.txt" 2>&1 &&
         timeout -k 10 300 python -u tools/ab_layout_forms.py >> "$O/ab_layout_forms.txt" 2>&1 ;;
    abl) timeout -k 10 300 python -u tools/ab_launch_form.py 10 > "$O/ab_launch_form.txt" 2>&1 ;;
    tct) for f in after before reference; do
             (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/tct_$f" -o run \
                 --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/training_call_trace.py" $f 20 \
                 > "$GRAFT_REPO_ROOT/$O/tct_$f.log" 2>&1) || exit 1
         done ;;
    benchab) for i in 1 2; do for o in first last; do
               timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 --side-legs $o \
                   > "$O/bench_${o}_$i.json" 2> "$O/bench_${o}_$i.err" || exit 1; done; done ;;
    gap) timeout -k 10 300 python -u tools/ab_bench_gap.py > "$O/ab_bench_gap.txt" 2>&1 &&
         timeout -k 10 300 python -u tools/ab_bench_gap.py >> "$O/ab_bench_gap.txt" 2>&1 ;;
    clock) timeout -k 10 300 python -u tools/clock_state.py 24 > "$O/clock_state.txt" 2>&1 ;;
    stampsw) for w in 0 20 0 20; do
               PCM_HIP_LIB=$PWD/3d-pointcloudreconstruction_amd/lib/libpcm_hip_stamps.so \
               PCM_HIP_TUNE_LIB=$PWD/3d-pointcloudreconstruction_amd/lib/libpcm_hip_stamps.so STAMP_WARM=$w \
                   timeout -k 10 300 python -u tools/stamp_filt.py fused 15 >> "$O/stamps_warm_cold.txt" 2>&1 || exit 1
             done ;;
    tctg) for f in after before; do
             (cd /tmp && TCT_GRAPH=5 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/tctg_$f" -o run \
                 --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/training_call_trace.py" $f 20 \
                 > "$GRAFT_REPO_ROOT/$O/tctg_$f.log" 2>&1) || exit 1
         done ;;
    benchv) for r in 1 2 3; do for v in ${BENCH_VARIANTS:-15 14 7}; do
               timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-emd --no-dense \
                   --no-icp --no-ref-call --tune-variant $v >> "$O/bench_variants.jsonl" 2>> "$O/bench_variants.err" || exit 1
           done; done ;;
    bench3) for r in 1 2 3; do
              timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench_$r.json" 2> "$O/bench_$r.err" || exit 1
            done ;;
    pmcf) (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d "$GRAFT_REPO_ROOT/$O/pmcf_fetch" -o fetch \
               --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/profile_kernels.py" fused ${PMC_VARIANTS:-7,16} \
               > "$GRAFT_REPO_ROOT/$O/pmcf_fetch.log" 2>&1 &&
           timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d "$GRAFT_REPO_ROOT/$O/pmcf_write" -o write \
               --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/profile_kernels.py" fused ${PMC_VARIANTS:-7,16} \
               > "$GRAFT_REPO_ROOT/$O/pmcf_write.log" 2>&1 &&
           timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/pmcf_kt" -o kt \
               --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/profile_kernels.py" fused ${PMC_VARIANTS:-7,16} \
               > "$GRAFT_REPO_ROOT/$O/pmcf_kt.log" 2>&1) ;;
    emdwarm) timeout -k 10 120 python -u tools/emd_warm_probe.py 6 50 > "$O/emd_warm.txt" 2>&1 &&
             timeout -k 10 120 python -u tools/emd_warm_probe.py 6 200 >> "$O/emd_warm.txt" 2>&1 ;;
    probeev) timeout -k 10 300 python -u tools/probe_events.py > "$O/probe_events.txt" 2>&1 ;;
    *) echo "unknown step $S"; exit 2 ;;
    esac
    rc=$?
    echo "[gpu_run] $S rc=$rc $(date +%T)"
    if [ $rc -ne 0 ]; then exit $rc; fi
done
