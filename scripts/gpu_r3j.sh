# round-3 final build: kernel trace + PMC profile (scripts/profile.sh), the dense re-solve count of
# the forcing test's input (fixed counter), and bench.py at N=2 rehearsed on one GPU
# (two ranks on cuda:0, gloo; the shared early-stop flag in the abort leg)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
L=trifocal_pose_estimation_using_improved_gpuhc_amd/lib
bash scripts/profile.sh r3j || exit 1
HC_TRIFOCAL_LIB=$L/libhc_trifocal_luwork.so timeout -k 10 120 python scripts/lu_work.py --scaled > gpurun_out/r3j_lu_work_scaled.json 2>&1; rc=$?; cat gpurun_out/r3j_lu_work_scaled.json; [ $rc -eq 0 ] || exit $rc
HC_TRIFOCAL_LIB=$L/libhc_trifocal_luwork.so timeout -k 10 120 python scripts/lu_work.py > gpurun_out/r3j_lu_work.json 2>&1; rc=$?; cat gpurun_out/r3j_lu_work.json; [ $rc -eq 0 ] || exit $rc
HC_BENCH_DEVICE=0 HC_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 > gpurun_out/r3j_bench_n2.json 2> gpurun_out/r3j_bench_n2.err; rc=$?; cat gpurun_out/r3j_bench_n2.json; exit $rc
