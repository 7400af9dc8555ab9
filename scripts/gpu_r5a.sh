# round 5, first lease: GPU tests on the ring-check / test-hook build, then the
# bare `bench.py --gpus 2` rehearsal (bench.py starts its two ranks itself;
# both on cuda:0 over gloo, RCCL refuses two ranks on one GPU)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
T=${1:-r5a}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
HC_BENCH_DEVICE=0 HC_BENCH_BACKEND=gloo timeout -k 10 700 python3 bench.py --gpus 2 > gpurun_out/${T}_bench_n2_rehearsal.json 2> gpurun_out/${T}_bench_n2.err; rc=$?; echo "n2 rc=$rc"; cat gpurun_out/${T}_bench_n2_rehearsal.json; exit $rc
