# bench.py at N=2 rehearsed on one MI355X (two ranks on cuda:0 over gloo: RCCL refuses
# two ranks on one GPU); every leg runs, the abort leg maps the cross-rank device flag
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
T=${1:-r4d}
HC_BENCH_DEVICE=0 HC_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 > gpurun_out/${T}_bench_n2.json 2> gpurun_out/${T}_bench_n2.err; rc=$?; cat gpurun_out/${T}_bench_n2.json; exit $rc
