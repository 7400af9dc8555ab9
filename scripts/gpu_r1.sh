cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/r1_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --abort-samples 200 > gpurun_out/r1_bench.log 2>&1; echo "bench rc=$?"
fi
tail -5 gpurun_out/r1_pytest.log
tail -3 gpurun_out/r1_bench.log
