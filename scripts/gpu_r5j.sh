# round 5: time to the first good pose (config 3, reference semantics, 12 runs
# per build and round, 3 interleaved rounds) of the abort kernel's LU variants:
# p1 (groups of 4, two loops: pivot-lane stores, then the rows below), abe4
# (groups of 4 in the eligible rows' region with 32-B scratch windows), abc2
# (groups of 2 in the eligible rows' region, the tracking kernel's LU); the
# abort-mode parity tests on each variant first
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
T=${T:-r5j}
P=$GRAFT_REPO_ROOT/trifocal_pose_estimation_using_improved_gpuhc_amd/lib
for b in ${BUILDS:-abe4 abc2}; do
  HC_TRIFOCAL_LIB=$P/libhc_trifocal_$b.so timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread -k "abort or config3" > gpurun_out/${T}_parity_$b.log 2>&1; rc=$?; tail -1 gpurun_out/${T}_parity_$b.log; [ $rc -eq 0 ] || exit $rc
done
for r in 0 1 2; do
  for b in ${BASE:-p1} ${BUILDS:-abe4 abc2}; do
    HC_TRIFOCAL_LIB=$P/libhc_trifocal_$b.so timeout -k 10 120 python scripts/ttfp.py 12 > gpurun_out/${T}_tmp.json || exit 1
    python -c "import json,sys; d=json.load(open('gpurun_out/${T}_tmp.json')); d.update(build='$b', round=$r); print(json.dumps(d))" >> gpurun_out/${T}_ttfp.jsonl
  done
done
cat gpurun_out/${T}_ttfp.jsonl
