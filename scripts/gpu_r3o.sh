# round-3 build with the packed dH/dx entries, merged dH/dt|H pass and the leaner back
# substitution: every GPU test, the full bench line, kernel trace + PMC profile
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r3o_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r3o_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py > gpurun_out/r3o_bench.json 2> gpurun_out/r3o_bench.err; rc=$?; cat gpurun_out/r3o_bench.json; [ $rc -eq 0 ] || exit $rc
bash scripts/profile.sh r3o || exit 1
L=trifocal_pose_estimation_using_improved_gpuhc_amd/lib
timeout -k 10 400 python scripts/ab_track.py HTH=$L/libhc_trifocal_hth.so SB=$L/libhc_trifocal_sb.so SBG=$L/libhc_trifocal_sbg.so SBGF=$L/libhc_trifocal_sbgf.so --rounds 3 > gpurun_out/r3o_ab.jsonl 2>&1; rc=$?; cat gpurun_out/r3o_ab.jsonl; exit $rc
