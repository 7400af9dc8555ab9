cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/r9_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r9_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 ./scripts/rcp_check > gpurun_out/r9_rcp.json 2>&1; rc=$?; echo "rcp rc=$rc"; cat gpurun_out/r9_rcp.json; [ $rc -eq 0 ] || exit $rc
for w in 4 3; do
  HC_TRIFOCAL_MINWAVES=$w timeout -k 10 300 python scripts/ubench.py > gpurun_out/r9_ubench_w$w.json 2>gpurun_out/r9_ubench_w$w.err; rc=$?; echo "ubench w$w rc=$rc"; cat gpurun_out/r9_ubench_w$w.json; [ $rc -eq 0 ] || exit $rc
done
