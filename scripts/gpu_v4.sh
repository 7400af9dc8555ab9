# v4 bring-up: parity tests under HC_TRIFOCAL_KERNEL=v4, then component + tracker microbenchmarks v3 vs v4, bench line v4
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=$1
HC_TRIFOCAL_KERNEL=v4 timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_v4.log 2>&1; rc=$?; echo "pytest v4 rc=$rc"; tail -15 gpurun_out/${T}_pytest_v4.log; [ $rc -eq 0 ] || exit $rc
HC_TRIFOCAL_KERNEL=v3 timeout -k 10 300 python scripts/ubench.py > gpurun_out/${T}_ubench_v3.json; rc=$?; echo "ubench v3 rc=$rc"; cat gpurun_out/${T}_ubench_v3.json; [ $rc -eq 0 ] || exit $rc
HC_TRIFOCAL_KERNEL=v4 timeout -k 10 300 python scripts/ubench.py > gpurun_out/${T}_ubench_v4.json; rc=$?; echo "ubench v4 rc=$rc"; cat gpurun_out/${T}_ubench_v4.json; [ $rc -eq 0 ] || exit $rc
HC_TRIFOCAL_KERNEL=v4 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${T}_bench_v4.json 2>gpurun_out/${T}_bench_v4.err; rc=$?; echo "bench v4 rc=$rc"; cat gpurun_out/${T}_bench_v4.json; [ $rc -eq 0 ] || exit $rc
