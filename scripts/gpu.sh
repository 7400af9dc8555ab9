# One runner for every GPU-box recipe (replaces rounds 3-5's one-off gpu_r*.sh;
# they are in the git history).  Run through gpurun from the repo root:
#   gpurun -- bash scripts/gpu.sh STEP[,STEP...] TAG [args]
# Steps (each under its own time limit; the chain stops at the first failure,
# and nothing more touches the GPU after it):
#   tests     pytest -m gpu                          -> gpurun_out/TAG_pytest.log
#   smoke     __graft_entry__.smoke()
#   luwork    LU work of the HC_DIAG_LUWORK build    -> TAG_lu_work.json
#   bench     the default bench line                 -> TAG_bench.json
#   profile   kernel trace + PMC passes + summary    -> TAG_pmc_summary.json, TAG_kernel_stats.csv
#   traffic   kernel trace + FETCH/WRITE passes only -> TAG_pmc_summary.json
#   datasets  held-out datasets (scripts/datasets.py)-> TAG_datasets.jsonl
#   n2        bare `bench.py --gpus 2` rehearsal, both ranks on cuda:0 -> TAG_bench_n2_rehearsal.json
#   ab        interleaved A/B of builds: extra args NAME=lib/libX.so ... (package-relative)
#   ttfp_ab   time to the first pose of builds NAME=lib/libX.so ... (package-relative): the abort-mode
#             parity tests on each, then 3 interleaved rounds of scripts/ttfp.py (config 3 in both
#             semantics, 12 runs each; the lone sample, 12 runs)      -> TAG_ttfp.jsonl
#   phases    per-phase cycles of the HC_DIAG_PHASES build (scripts/diag_phases.py)
#   stress    time slicing under concurrent streams (scripts/slice_stress.py: 4 cold, 4 warm, 8 cold)
#   validate  tests,luwork,bench,profile,datasets
# Extra environment: BENCH_ARGS (bench step), AB_ROUNDS (ab step, default 3), AB_ARGS (more ab_track.py options), TTFP_ARGS (ttfp_ab step,
# e.g. "--dataset 10").
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
STEPS=$1; T=$2; shift 2
O=gpurun_out
L=$PWD/trifocal_pose_estimation_using_improved_gpuhc_amd/lib
P=$PWD/trifocal_pose_estimation_using_improved_gpuhc_amd
mkdir -p $O
[ "$STEPS" = validate ] && STEPS=tests,luwork,bench,profile,datasets
ver() { python -c 'import sys; sys.path.insert(0,"."); from trifocal_pose_estimation_using_improved_gpuhc_amd import _abi; print(_abi.build_id())'; }
run() {   # run NAME SECONDS CMD...: one GPU step under its own limit
  local n=$1 s=$2; shift 2
  echo "[$n] $(date +%T) start" >&2
  timeout -k 10 $s "$@"; local rc=$?
  echo "[$n] $(date +%T) rc=$rc" >&2
  return $rc
}
for step in ${STEPS//,/ }; do
  case $step in
    tests) run tests 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/${T}_pytest.log 2>&1; rc=$?; tail -3 $O/${T}_pytest.log ;;
    smoke) run smoke 300 python -c 'import __graft_entry__ as g; g.smoke()'; rc=$? ;;
    luwork) HC_TRIFOCAL_LIB=$L/libhc_trifocal_luwork.so run luwork 200 python scripts/lu_work.py > $O/${T}_lu_work.json; rc=$?; cat $O/${T}_lu_work.json ;;
    bench) run bench 600 python bench.py $BENCH_ARGS > $O/${T}_bench.json 2> $O/${T}_bench.err; rc=$?; cat $O/${T}_bench.json ;;
    profile|traffic)
      B="python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-small-launch --abort-samples 0 --noisy-trials 0 --streams 1 --pipelined-streams 0"
      run trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_trace -o run -- $B > $O/${T}_trace.log 2>&1; rc=$?
      if [ $step = profile ]; then
        SETS=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY"
              "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
              "SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_LDS SQ_IFETCH"
              "FETCH_SIZE" "WRITE_SIZE")
      else
        SETS=("FETCH_SIZE" "WRITE_SIZE")
      fi
      i=0
      for set in "${SETS[@]}"; do
        [ $rc -eq 0 ] || break
        i=$((i+1))
        run pmc$i 300 rocprofv3 --pmc $set --output-format csv -d $O/${T}_pmc$i -o run -- $B > $O/${T}_pmc$i.log 2>&1; rc=$?
      done
      if [ $rc -eq 0 ]; then
        python scripts/pmc_summary.py $T $O/${T}_pmc_summary.json > /dev/null; rc=$?
        cp $O/${T}_trace/run_kernel_stats.csv $O/${T}_kernel_stats.csv
      fi ;;
    datasets) run datasets 900 python scripts/datasets.py $L/libhc_trifocal_luwork.so "$@" > $O/${T}_datasets.jsonl; rc=$?; cat $O/${T}_datasets.jsonl ;;
    n2) HC_BENCH_DEVICE=0 HC_BENCH_BACKEND=gloo run n2 700 python3 bench.py --gpus 2 > $O/${T}_bench_n2_rehearsal.json 2> $O/${T}_bench_n2.err; rc=$?; cat $O/${T}_bench_n2_rehearsal.json ;;
    ab)
      args=""; last=""
      for kv in "$@"; do args="$args ${kv%%=*}=$P/${kv#*=}"; last=$P/${kv#*=}; done
      HC_TRIFOCAL_LIB=$last run ab_parity 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread -k "not cli" > $O/${T}_parity.log 2>&1; rc=$?; tail -3 $O/${T}_parity.log
      [ $rc -eq 0 ] && { run ab 900 python -u scripts/ab_track.py $args --rounds ${AB_ROUNDS:-3} $AB_ARGS > $O/${T}_ab.jsonl; rc=$?; cat $O/${T}_ab.jsonl; } ;;
    ttfp_ab)
      rc=0
      for kv in "$@"; do
        HC_TRIFOCAL_LIB=$P/${kv#*=} run parity_${kv%%=*} 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread -k "abort or config3 or row_permuted" > $O/${T}_parity_${kv%%=*}.log 2>&1; rc=$?; tail -1 $O/${T}_parity_${kv%%=*}.log
        [ $rc -eq 0 ] || break
      done
      for rd in 0 1 2; do
        [ $rc -eq 0 ] || break
        for kv in "$@"; do
          for mode in "" "--inflight" "--samples 1"; do
            HC_TRIFOCAL_LIB=$P/${kv#*=} run ttfp 120 python scripts/ttfp.py 12 $mode $TTFP_ARGS > $O/${T}_tmp.json; rc=$?
            [ $rc -eq 0 ] || break 2
            python -c "import json,sys; d=json.load(open('$O/${T}_tmp.json')); d.update(build='${kv%%=*}', round=$rd); print(json.dumps(d))" >> $O/${T}_ttfp.jsonl
          done
        done
      done
      [ -f $O/${T}_ttfp.jsonl ] && python -c "
import json,collections
g=collections.defaultdict(list)
for l in open('$O/${T}_ttfp.jsonl'):
    d=json.loads(l); g[(d['build'],d['samples'],d['inflight_stop'])].append(d['median'])
for k,v in sorted(g.items()): print(k, v)" ;;
    phases) HC_TRIFOCAL_LIB=$L/libhc_trifocal_phases.so run phases 300 python scripts/diag_phases.py > $O/${T}_phases.json; rc=$?; cat $O/${T}_phases.json ;;
    stress)
      run stress4 300 python scripts/slice_stress.py $O/${T}_stress4.jsonl 4 4 > /dev/null 2>&1; rc=$?
      [ $rc -eq 0 ] && { run stress4w 300 python scripts/slice_stress.py $O/${T}_stress4w.jsonl 4 4 --warm-streams > /dev/null 2>&1; rc=$?; }
      [ $rc -eq 0 ] && { run stress8 300 python scripts/slice_stress.py $O/${T}_stress8.jsonl 8 3 > /dev/null 2>&1; rc=$?; } ;;
    *) echo "unknown step $step"; rc=2 ;;
  esac
  [ $rc -eq 0 ] || { echo "step $step failed (rc=$rc): stopping"; exit $rc; }
done
echo "build $(ver)"
