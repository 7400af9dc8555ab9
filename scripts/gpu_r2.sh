cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/r2_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r2_pytest.log | tail -2
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python scripts/ubench.py > gpurun_out/r2_ubench.json 2> gpurun_out/r2_ubench.err; echo "ubench rc=$?"; cat gpurun_out/r2_ubench.json
rocprofv3 -L > gpurun_out/r2_counters.txt 2>&1; echo "list rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r2 -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --abort-samples 0 > gpurun_out/r2_bench_prof.log 2>&1; echo "prof rc=$?"
find gpurun_out/prof_r2 -name "*stats*" | head
