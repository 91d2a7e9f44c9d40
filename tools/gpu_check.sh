#!/bin/bash
# One gpurun session: GPU parity tests, kernel sweep, bench, rocprofv3 kernel-trace stats and PMC HBM-traffic passes.
#   gpurun --timeout 1200 -- bash tools/gpu_check.sh <tag> [steps...]
# steps: tests testsdyn testfile testfiles piab fsab d16ab rawab pmcall kbench bench jitter export shape125 configs coloab dynab hllab cut0ab buildtrace profk125 prof profk pmc pmck variants (default: tests kbench bench prof pmc)
# KBENCH_ONLY=name,name restricts the kbench sweeps (KBENCH_ARGS: extra kbench flags for variants, KBENCH_TAG: log suffix); variants = every build/variants/libesgpu_*.so via ESGPU_LIBRARY.  Every GPU step has its own time limit; the first failure ends it.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r1}
shift || true
STEPS=${*:-tests kbench bench prof pmc}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name seconds cmd...
    local name=$1 secs=$2
    shift 2
    echo "== $name $(date +%T)"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc $(date +%T)"
    tail -5 "$OUT/$name.log"
    [ $rc -eq 0 ] || exit $rc
}
for s in $STEPS; do
    case $s in
        tests) run pytest_gpu 1100 python3 -u -m pytest "$R/tests" -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
        kbench) run kbench 600 python3 "$R/tools/kbench.py" --docs 1000000000 --reps 5 ${KBENCH_ONLY:+--only $KBENCH_ONLY} ;;
        bench) run bench 600 python3 "$R/bench.py" ;;
        jitter) for j in 0 60000 3600000; do
                    run "kbench_jitter_$j" 300 python3 "$R/tools/kbench.py" --docs 1000000000 --reps 5 --ts-jitter $j \
                        --only north_star,config2_dh_ext,date_hist,terms_dh || exit 1
                done ;;
        export) run export_bench 300 python3 "$R/tools/export_bench.py" --docs 250000000 --reps 3 ;;
        shape125) run kbench_125m 300 python3 "$R/tools/kbench.py" --docs 125000000 --reps 5 --shards 8 ;;
        configs) # every BASELINE config at its own shape (1 GPU: the 8 shards of configs 3-5 collected in turn)
              run bench_config2 300 python3 "$R/bench.py" --workload config2 --docs 100000000 --cpu-docs 160000000 &&
              run bench_config3 300 python3 "$R/bench.py" --workload config3 --shards 8 --docs 125000000 --cpu-docs 320000000 &&
              run bench_config4 300 python3 "$R/bench.py" --workload config4 --shards 8 --docs 125000000 --cpu-docs 320000000 &&
              run bench_config5 300 python3 "$R/bench.py" --workload config5 --shards 8 --docs 125000000 --cpu-docs 320000000 &&
              run bench_ns_shards8 300 python3 "$R/bench.py" --shards 8 --docs 125000000 --cpu-docs 0 ;;
        coloab) # co-located reduce (one build_reduce call per request) vs one build per shard + host reduce (--no-colo)
              for i in 1 2; do for c in "" "--no-colo"; do
                  t=${c:+_nocolo}
                  run "bench_ns8${t}_$i" 300 python3 "$R/bench.py" --shards 8 --docs 125000000 --cpu-docs 0 $c || exit 1
                  run "bench_c5${t}_$i" 300 python3 "$R/bench.py" --workload config5 --shards 8 --docs 125000000 --cpu-docs 0 $c || exit 1
              done; done ;;
        colotrace) # per-phase host marks of build_reduce (and each skeleton build) in the 8-shard north star / config 5
              ESGPU_TRACE_BUILD=1 run bench_ns8_colotrace 300 python3 "$R/bench.py" --shards 8 --docs 125000000 --cpu-docs 0 \
                  --steps 4 --warmup 2 &&
              run bench_ns8 300 python3 "$R/bench.py" --shards 8 --docs 125000000 --cpu-docs 0 &&
              run bench_c5 300 python3 "$R/bench.py" --workload config5 --shards 8 --docs 125000000 --cpu-docs 0 ;;
        schemes) # pipelined-phase A/B on one box: rotating plans vs one plan per shard
              for i in 1 2; do for sc in rotate sets; do
                  run "bench_ns8_${sc}_$i" 300 python3 "$R/bench.py" --shards 8 --docs 125000000 --cpu-docs 0 --scheme $sc || exit 1
                  run "bench_c5_${sc}_$i" 300 python3 "$R/bench.py" --workload config5 --shards 8 --docs 125000000 --cpu-docs 0 --scheme $sc || exit 1
              done; done ;;
        dynab) # collect kernel: static block ranges vs dynamic chunk claiming (ESGPU_DYN), 125M- and 1B-doc shards
              for i in 1 2; do for d in 0 1; do
                  ESGPU_DYN=$d run "kbench_125m_dyn${d}_$i" 300 python3 "$R/tools/kbench.py" --docs 125000000 --reps 5 \
                      ${KBENCH_ONLY:+--only $KBENCH_ONLY} || exit 1
              done; done
              for d in 0 1; do
                  ESGPU_DYN=$d run "kbench_1b_dyn$d" 300 python3 "$R/tools/kbench.py" --docs 1000000000 --reps 5 \
                      ${KBENCH_ONLY:+--only $KBENCH_ONLY} || exit 1
              done ;;
        hllab) # HLL register phases: raises logged for a gather (default) vs one global atomicMax per raise (ESGPU_HLL_LOG=0)
              for d in 1 0; do for docs in 125000000 1000000000; do
                  ESGPU_HLL_LOG=$d run "kbench_hll${d}_$docs" 300 python3 "$R/tools/kbench.py" --docs $docs --reps 5 \
                      --only config4_card || exit 1
              done; done ;;
        fsab) # HLL floored stream (one pass + gather + tail) vs the register phases (ESGPU_HLL_FS=0)
              for f in 1 0; do for docs in 125000000 1000000000; do
                  ESGPU_HLL_FS=$f run "kbench_fs${f}_$docs" 300 python3 "$R/tools/kbench.py" --docs $docs --reps 5 \
                      --only config4_card || exit 1
              done; done ;;
        gatherab) # config 4 at one fresh 125M plan: HLL tests, kbench, and the rocprof kernel trace of the request
              run pytest_hll 600 python3 -u -m pytest "$R/tests/test_gpu_hll_floor.py" "$R/tests/test_gpu_parity.py" -k "card or hll or floor" \
                  -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread || exit 1
              for i in 1 2; do
                  run "kbench_c4_125m_$i" 300 python3 "$R/tools/kbench.py" --docs 125000000 --reps 7 --only config4_card || exit 1
              done
              cd /tmp && run rocprof_c4 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profc4" -o kb -- \
                  python3 "$R/tools/kbench.py" --docs 125000000 --reps 3 --only config4_card ;;
        d16ab) # 16-bit deltas (packed cells' metric, range predicates) vs 32-bit (ESGPU_D16=0), same box
              for d in 1 0; do
                  ESGPU_D16=$d run "kbench_d16_$d" 400 python3 "$R/tools/kbench.py" --docs 1000000000 --reps 5 \
                      --only ${KBENCH_ONLY:-north_star,ns_avg,config5,config1_terms_stats} || exit 1
              done ;;
        rawab) # histogram-only raw-load kernels (VK bit 1024) vs the converting loader (ESGPU_RAW_HIST=0), same box
              for r in 1 0; do
                  ESGPU_RAW_HIST=$r run "kbench_raw_$r" 400 python3 "$R/tools/kbench.py" --docs 1000000000 --reps 5 \
                      --only ${KBENCH_ONLY:-date_hist,config2_dh_ext} || exit 1
              done ;;
        cut0ab) # HLL phase 0 length (ESGPU_HLL_CUT0 x 2^p values through the partitioned phase 0)
              for c in 4 16 64; do for docs in 125000000 1000000000; do
                  ESGPU_HLL_CUT0=$c run "kbench_cut${c}_$docs" 300 python3 "$R/tools/kbench.py" --docs $docs --reps 5 \
                      --only config4_card || exit 1
              done; done ;;
        testsdyn) ESGPU_DYN=1 run pytest_gpu_dyn 1100 python3 -u -m pytest "$R/tests" -m gpu -x -v -p no:cacheprovider \
                      --timeout 300 --timeout-method thread ;;
        buildtrace) # per-phase host marks of every shard build (ESGPU_TRACE_BUILD) in the 8-shard north star
              ESGPU_TRACE_BUILD=1 run bench_ns8_trace 300 python3 "$R/bench.py" --shards 8 --docs 125000000 --cpu-docs 0 \
                  --steps 4 --warmup 2 ;;
        prof) cd /tmp && run rocprof_stats 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- \
                  python3 "$R/bench.py" --steps 10 --warmup 3 --cpu-docs 0 --inflight 1 ;;
        c3) # config 3 at 125M docs: clean (postings form) and with 1 % deletions (scatter form), kernel and bench line
              run kbench_c3_125m 300 python3 "$R/tools/kbench.py" --docs 125000000 --reps 5 --only config3_url &&
              run kbench_c3_125m_del 300 python3 "$R/tools/kbench.py" --docs 125000000 --reps 5 --only config3_url --deletes 0.01 &&
              run bench_config3 300 python3 "$R/bench.py" --workload config3 --shards 8 --docs 125000000 --cpu-docs 0 ;;
        hot16ab) # config 3 postings hot pass: 32-bit recoded column vs the 16-bit hot-slot column, clean and 1 % deleted
              for h in 0 1; do for d in 0 0.01; do
                  ESGPU_HOT16=$h run "kbench_c3_hot16_${h}_del$d" 300 python3 "$R/tools/kbench.py" --docs 125000000 --reps 7 \
                      --only config3_url --deletes $d || exit 1
              done; done ;;
        compactab) # compact columns (16-bit ordinals, 32-bit timestamp deltas) vs the upload-width columns
              for c in 1 0; do for docs in 1000000000 125000000; do
                  ESGPU_COMPACT=$c run "kbench_compact${c}_$docs" 400 python3 "$R/tools/kbench.py" --docs $docs --reps 5 \
                      --only terms_host,date_hist,config2_dh_ext,terms_dh,config1_terms_stats,north_star,config5,dh_terms,heatmap || exit 1
              done; done ;;
        smoke) run smoke 300 python3 -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" ;;
        inflightab) # requests in flight: 2 / 3 / 4 (north star 1 x 1B and 8 x 125M)
              for d in 2 3 4; do
                  run "bench_if$d" 300 python3 "$R/bench.py" --inflight $d --cpu-docs 0 || exit 1
                  run "bench_ns8_if$d" 300 python3 "$R/bench.py" --inflight $d --shards 8 --docs 125000000 --cpu-docs 0 || exit 1
              done ;;
        proftl) # kernel timeline of the default bench (2 requests in flight): GPU idle gaps between collect launches
              cd /tmp && run rocprof_timeline 600 rocprofv3 --kernel-trace --output-format csv -d "$OUT/proftl" -o bench -- \
                  python3 "$R/bench.py" --steps 10 --warmup 3 --cpu-docs 0 ;;
        profk) cd /tmp && run rocprof_kbench 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profk" -o kbench -- \
                   python3 "$R/tools/kbench.py" --docs 1000000000 --reps 3 ;;
        profk125) cd /tmp && run rocprof_kbench125 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profk125" -o kb125 -- \
                   python3 "$R/tools/kbench.py" --docs 125000000 --reps 3 ${KBENCH_ONLY:+--only $KBENCH_ONLY} ;;
        testfiles) # several test files in one pytest process: TESTFILES="test_gpu_layouts test_gpu_hotcold"
              args=""; for f in ${TESTFILES:-test_gpu_parity}; do args="$args $R/tests/$f.py"; done
              run pytest_files 900 python3 -u -m pytest $args -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
        piab) # packed integer metric cells (ESGPU_PI) and lane-rotated copies of their count + sum words (ESGPU_PI_COPIES)
              for pi in 1 0; do
                  ESGPU_PI=$pi run "kbench_pi$pi" 400 python3 "$R/tools/kbench.py" --docs 1000000000 --reps 5 \
                      --only ${KBENCH_ONLY:-north_star,ns_avg,config5,config1_terms_stats} || exit 1
              done
              for c in 2 3; do
                  ESGPU_PI_COPIES=$c run "kbench_picp$c" 400 python3 "$R/tools/kbench.py" --docs 1000000000 --reps 5 \
                      --only ${KBENCH_ONLY:-north_star,ns_avg,config5,config1_terms_stats} || exit 1
              done ;;
        replayab) # breadth-first replay of terms(host){terms(url)}: compacted winners' docs vs one pass per batch
              for c in 1 0; do for docs in 125000000 1000000000; do
                  ESGPU_REPLAY_COMPACT=$c run "kbench_replay${c}_$docs" 400 python3 "$R/tools/kbench.py" --docs $docs --reps 3 \
                      --only hosts_urls || exit 1
              done; done ;;
        c3stats) # config 3: the per-segment statistics build (bench precomputed) and the filtered / deleted forms
              run bench_config3 300 python3 "$R/bench.py" --workload config3 --shards 8 --docs 125000000 --cpu-docs 0 --steps 5 &&
              run kbench_c3_125m_del 300 python3 "$R/tools/kbench.py" --docs 125000000 --reps 5 --only config3_url --deletes 0.01 ;;
        profreplay) # kernel breakdown of the breadth-first replay (terms(host){terms(url)} at 1B docs)
              cd /tmp && run rocprof_replay 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profreplay" -o kb -- \
                  python3 "$R/tools/kbench.py" --docs 1000000000 --reps 2 --only hosts_urls ;;
        testfile) run "pytest_${TESTFILE:-x}" 600 python3 -u -m pytest "$R/tests/${TESTFILE:-test_gpu_parity}.py" -m gpu -x -v \
                      -p no:cacheprovider --timeout 300 --timeout-method thread ;;
        pmc) cd /tmp && run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_fetch" -o bench -- \
                 python3 "$R/bench.py" --steps 3 --warmup 1 --cpu-docs 0 --inflight 1 &&
             run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_write" -o bench -- \
                 python3 "$R/bench.py" --steps 3 --warmup 1 --cpu-docs 0 --inflight 1 ;;
        pmcall) # FETCH_SIZE / WRITE_SIZE passes (one counter per pass) of every bench shape's collect, 4 collects each
                # (kbench --reps 3), for tools/pmc_traffic.py -> profiles/hbm_traffic.json (bench roofline.traffic)
              for spec in north_star:1000000000 north_star:125000000 config2_dh_ext:100000000 config3_url:125000000 \
                          config4_card:125000000 config5:125000000; do
                  v=${spec%%:*}; d=${spec##*:}
                  for c in FETCH_SIZE WRITE_SIZE; do
                      cd /tmp && run "pmcall_${v}_${d}_$c" 300 rocprofv3 --pmc $c --kernel-trace --output-format csv \
                          -d "$OUT/pmcall_${v}_${d}_$c" -o kb -- python3 "$R/tools/kbench.py" --docs $d --reps 3 --only $v \
                          || exit 1
                  done
              done ;;
        pmck) # counters for the kbench shapes in KBENCH_ONLY (default config3_url), one counter group per pass
              for grp in FETCH_SIZE WRITE_SIZE "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
                         "SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
                  tag=$(echo "$grp" | cut -d' ' -f1)
                  cd /tmp && run "pmck_$tag" 600 rocprofv3 --pmc $grp --kernel-trace --output-format csv \
                      -d "$OUT/pmck_$tag" -o kb -- python3 "$R/tools/kbench.py" --docs 1000000000 --reps 1 \
                      --only "${KBENCH_ONLY:-config3_url}"
              done ;;
        variants) for so in "$R"/build/variants/libesgpu_*.so; do
                      v=$(basename "$so" .so)
                      ESGPU_LIBRARY=$so run "kbench_$v${KBENCH_TAG:-}" 600 python3 "$R/tools/kbench.py" --docs 1000000000 --reps 5 \
                          ${KBENCH_ONLY:+--only $KBENCH_ONLY} ${KBENCH_ARGS:-}
                  done ;;
        ranksim) # per-rank host time of esgpu_comm_build_reduce, 8 in-process ranks on this GPU, 125M docs per rank
              for w in ${RANKSIM_ONLY:-north_star config3 config4 config5}; do
                  run "ranksim_$w" 300 python3 "$R/tools/rank_sim.py" --workload $w --ranks 8 --docs 125000000 --reqs 20 || exit 1
              done ;;
        *) echo "unknown step $s"; exit 2 ;;
    esac
done
echo "== done"
