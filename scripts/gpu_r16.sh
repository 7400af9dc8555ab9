cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/r16_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r16_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 ./scripts/lu_bench 200 > gpurun_out/r16_lu.json; rc=$?; echo "lu rc=$rc"; cat gpurun_out/r16_lu.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/ubench.py > gpurun_out/r16_ubench.json; rc=$?; echo "ubench rc=$rc"; cat gpurun_out/r16_ubench.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r16_bench.json 2>gpurun_out/r16_bench.err; rc=$?; echo "bench rc=$rc"; cat gpurun_out/r16_bench.json; [ $rc -eq 0 ] || exit $rc
