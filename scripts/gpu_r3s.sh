# round-3 final build (packed dH/dx, merged and balanced dH/dt|H, gather offsets, lean back
# substitution): every GPU test, the full bench line, kernel trace + PMC profile
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r3s_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r3s_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py > gpurun_out/r3s_bench.json 2> gpurun_out/r3s_bench.err; rc=$?; cat gpurun_out/r3s_bench.json; [ $rc -eq 0 ] || exit $rc
bash scripts/profile.sh r3s
