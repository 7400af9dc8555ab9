# round-3 final build after LU column groups of 2 (dea2602): every GPU test, bench line, trace + PMC
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r3x_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r3x_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py > gpurun_out/r3x_bench.json 2> gpurun_out/r3x_bench.err; rc=$?; cat gpurun_out/r3x_bench.json; [ $rc -eq 0 ] || exit $rc
bash scripts/profile.sh r3x
