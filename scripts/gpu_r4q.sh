# time to the first good pose (config 3, reference semantics, 12 runs per round)
# of v9.6 (r4j), v9.7 (r4p: fused group tests in every kernel) and split (v9.7
# with the abort kernel's groups of 4 unfused), 3 interleaved rounds; parity of
# the abort-mode tests on split first
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
P=$GRAFT_REPO_ROOT/trifocal_pose_estimation_using_improved_gpuhc_amd/lib
HC_TRIFOCAL_LIB=$P/libhc_trifocal_split.so timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread -k "abort or config3" > gpurun_out/r4q_parity.log 2>&1; rc=$?; tail -2 gpurun_out/r4q_parity.log; [ $rc -eq 0 ] || exit $rc
for r in 0 1 2; do
  for b in r4j r4p split; do
    HC_TRIFOCAL_LIB=$P/libhc_trifocal_$b.so timeout -k 10 120 python scripts/ttfp.py 12 > gpurun_out/r4q_tmp.json || exit 1
    python -c "import json,sys; d=json.load(open('gpurun_out/r4q_tmp.json')); d.update(build='$b', round=$r); print(json.dumps(d))" >> gpurun_out/r4q_ttfp.jsonl
  done
done
cat gpurun_out/r4q_ttfp.jsonl
