# back substitution with an unmasked rhs update (rows at or below position I are already solved,
# so their rhs is dead): interleaved A/B against HEAD
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
L=trifocal_pose_estimation_using_improved_gpuhc_amd/lib
timeout -k 10 900 python scripts/ab_track.py HEAD=$L/libhc_trifocal.so UB=$L/libhc_trifocal_ub.so --rounds 4 > gpurun_out/r3aa_ab.jsonl 2>&1; rc=$?; cat gpurun_out/r3aa_ab.jsonl; exit $rc
