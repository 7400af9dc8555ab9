# round 5: the bare `bench.py --gpus 2` rehearsal (fixed), then the A/B of the
# eligible-rows LU groups (v1: pivot lane to the buffer, v2: scratch windows)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
T=${T:-r5c}
HC_BENCH_DEVICE=0 HC_BENCH_BACKEND=gloo timeout -k 10 700 python3 bench.py --gpus 2 > gpurun_out/${T}_bench_n2_rehearsal.json 2> gpurun_out/${T}_bench_n2.err; rc=$?; echo "n2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab.sh r5c base=lib/libhc_trifocal_r5base.so v1=lib/libhc_trifocal_v1.so v2=lib/libhc_trifocal_v2.so
