# LU column groups of 1 for the first 4 / 8 / 14 pivot steps (2 after): interleaved A/B against HEAD
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
L=trifocal_pose_estimation_using_improved_gpuhc_amd/lib
timeout -k 10 900 python scripts/ab_track.py HEAD=$L/libhc_trifocal.so O4=$L/libhc_trifocal_o4.so O8=$L/libhc_trifocal_o8.so O14=$L/libhc_trifocal_o14.so --rounds 3 > gpurun_out/r3z_ab.jsonl 2>&1; rc=$?; cat gpurun_out/r3z_ab.jsonl; exit $rc
