# round 5: the bare `bench.py --gpus 2` rehearsal on the shipped build
# (bench.py starts its two ranks; both on cuda:0 over gloo)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
T=${1:-r5z}
HC_BENCH_DEVICE=0 HC_BENCH_BACKEND=gloo timeout -k 10 700 python3 bench.py --gpus 2 > gpurun_out/${T}_bench_n2_rehearsal.json 2> gpurun_out/${T}_bench_n2.err; rc=$?; echo "n2 rc=$rc"; cat gpurun_out/${T}_bench_n2_rehearsal.json; exit $rc
