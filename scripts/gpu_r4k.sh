# the config-3 test with every tracked path checked against the oracle
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -x -v -m gpu --timeout 300 --timeout-method thread -k config3 > gpurun_out/r4k_config3.log 2>&1; rc=$?; tail -5 gpurun_out/r4k_config3.log; exit $rc
