# round-3 final build (LU groups of 2, unmasked back-substitution update): every GPU test, bench line, trace + PMC
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r3ab_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r3ab_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py > gpurun_out/r3ab_bench.json 2> gpurun_out/r3ab_bench.err; rc=$?; cat gpurun_out/r3ab_bench.json; [ $rc -eq 0 ] || exit $rc
bash scripts/profile.sh r3ab
