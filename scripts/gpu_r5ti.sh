# round 5: the tie steps (18, 19, 21, 22) skip their lowest-position
# reduction when the solve has no tie there (tie1) against v10.2
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
bash scripts/gpu_ab.sh r5ti v102=lib/libhc_trifocal_v102.so tie1=lib/libhc_trifocal_tie1.so
