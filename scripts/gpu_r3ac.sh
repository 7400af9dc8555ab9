# pivot search: the rare-path test as one SGPR value ((popcount ^ 2) | bad_lo | bad_hi, one compare)
# instead of the compiler's cselect chain, now that the back substitution has no exec region:
# interleaved A/B against HEAD
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
L=trifocal_pose_estimation_using_improved_gpuhc_amd/lib
timeout -k 10 900 python scripts/ab_track.py HEAD=$L/libhc_trifocal.so RT=$L/libhc_trifocal_rt.so --rounds 4 > gpurun_out/r3ac_ab.jsonl 2>&1; rc=$?; cat gpurun_out/r3ac_ab.jsonl; exit $rc
