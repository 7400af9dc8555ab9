cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
# v2 (default) parity
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/r4_pytest_v2.log 2>&1; rc=$?
echo "pytest v2 rc=$rc"; grep -E "passed|failed|Error" gpurun_out/r4_pytest_v2.log | tail -6
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
# v1 parity
HC_TRIFOCAL_KERNEL=v1 timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/r4_pytest_v1.log 2>&1; rc=$?
echo "pytest v1 rc=$rc"; grep -E "passed|failed|Error" gpurun_out/r4_pytest_v1.log | tail -6
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for cfg in "v1 2" "v2 2" "v2 3"; do set -- $cfg
  HC_TRIFOCAL_KERNEL=$1 HC_TRIFOCAL_MINWAVES=$2 timeout -k 10 300 python scripts/ubench.py > gpurun_out/r4_ubench_$1_$2.json 2>/dev/null; rc=$?
  echo "ubench $1 $2 rc=$rc"; cat gpurun_out/r4_ubench_$1_$2.json
  if [ $rc -ne 0 ]; then exit $rc; fi
done
