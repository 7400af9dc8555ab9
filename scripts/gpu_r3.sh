cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/r3_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|Error" gpurun_out/r3_pytest.log | tail -8
