# round-3: full bench line of the final build + the dense re-solve count (HC_DIAG_LUWORK build)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python bench.py > gpurun_out/r3e_bench.json 2> gpurun_out/r3e_bench.err; rc=$?; echo "bench rc=$rc"; cat gpurun_out/r3e_bench.json; [ $rc -eq 0 ] || exit $rc
HC_TRIFOCAL_LIB=trifocal_pose_estimation_using_improved_gpuhc_amd/lib/libhc_trifocal_luwork.so timeout -k 10 200 python scripts/lu_work.py > gpurun_out/r3e_lu_work.json 2>&1; rc=$?; cat gpurun_out/r3e_lu_work.json; [ $rc -eq 0 ] || exit $rc
L=trifocal_pose_estimation_using_improved_gpuhc_amd/lib
timeout -k 10 300 python scripts/ab_track.py T3=$L/libhc_trifocal.so UM=$L/libhc_trifocal_xUM.so --rounds 3 > gpurun_out/r3e_ab.jsonl 2>&1; rc=$?; cat gpurun_out/r3e_ab.jsonl; exit $rc
