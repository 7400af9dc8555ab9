# final round-3 validation, short form: every GPU test and the bench line of HEAD, then the rare-test A/B
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r3ae_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r3ae_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py > gpurun_out/r3ae_bench.json 2> gpurun_out/r3ae_bench.err; rc=$?; cat gpurun_out/r3ae_bench.json; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r3ac.sh
