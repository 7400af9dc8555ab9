# LU column groups per pivot step: interleaved A/B of groups of 4 from step 12 / 20 / 24 on,
# or for the first 10 steps, against HEAD (groups of 2 everywhere); then the executed LU work
# of HEAD (HC_DIAG_LUWORK build) for bench.py's pricing
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
L=trifocal_pose_estimation_using_improved_gpuhc_amd/lib
HC_TRIFOCAL_LIB=$L/libhc_trifocal_luwork.so timeout -k 10 200 python scripts/lu_work.py > gpurun_out/r3y_lu_work.json 2>&1; rc=$?; cat gpurun_out/r3y_lu_work.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python scripts/ab_track.py HEAD=$L/libhc_trifocal.so S12=$L/libhc_trifocal_s12.so S20=$L/libhc_trifocal_s20.so S24=$L/libhc_trifocal_s24.so E10=$L/libhc_trifocal_e10.so --rounds 3 > gpurun_out/r3y_ab.jsonl 2>&1; rc=$?; cat gpurun_out/r3y_ab.jsonl; exit $rc
