cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/r6_pytest.log 2>&1; rc=$?; echo "pytest v3 rc=$rc"; tail -3 gpurun_out/r6_pytest.log; [ $rc -eq 0 ] || exit $rc
for cfg in "v3 3" "v3 4" "v2 3"; do
  set -- $cfg
  HC_TRIFOCAL_KERNEL=$1 HC_TRIFOCAL_MINWAVES=$2 timeout -k 10 300 python scripts/ubench.py > gpurun_out/r6_ubench_$1_$2.json 2>gpurun_out/r6_ubench_$1_$2.err; rc=$?; echo "ubench $1 $2 rc=$rc"; cat gpurun_out/r6_ubench_$1_$2.json; [ $rc -eq 0 ] || exit $rc
done
HC_TRIFOCAL_MINWAVES=4 timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/r6_pytest_w4.log 2>&1; rc=$?; echo "pytest v3 w4 rc=$rc"; tail -3 gpurun_out/r6_pytest_w4.log; [ $rc -eq 0 ] || exit $rc
