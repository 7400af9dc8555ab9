# round 5: per-step column-group liveness (HC_DIAG_LIVE build) on datasets 000/001/002
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
L=$GRAFT_REPO_ROOT/trifocal_pose_estimation_using_improved_gpuhc_amd/lib/libhc_trifocal_live.so
for d in 0 1 2; do
  HC_TRIFOCAL_LIB=$L timeout -k 10 120 python -u scripts/lu_live.py --dataset $d >> gpurun_out/r5lv_live.jsonl || exit $?
done
echo ok
