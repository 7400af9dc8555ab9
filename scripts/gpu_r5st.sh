# round 5: column groups by structural class (st1: provably dead groups
# untested, always-live groups unconditional; with the carried eligible mask)
# against el1 and the shipped build (base6); pr1 = st1 with consecutive
# always-live groups stored / read as pairs (one wait)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
bash scripts/gpu_ab.sh r5st2 base6=lib/libhc_trifocal_base6.so el1=lib/libhc_trifocal_el1.so pr1=lib/libhc_trifocal_pr1.so st1=lib/libhc_trifocal_st1.so
