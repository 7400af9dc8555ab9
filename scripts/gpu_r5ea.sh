# round 5: the evaluations' operand look-ahead depth (EV_AHEAD 1 / 3 against
# the shipped 2) re-checked on v10.2
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
bash scripts/gpu_ab.sh r5ea v102=lib/libhc_trifocal_v102.so ea1=lib/libhc_trifocal_ea1.so ea3=lib/libhc_trifocal_ea3.so
