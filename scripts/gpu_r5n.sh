# round 5: the multiplier in the eligible rows' region (p4) against v9.9 (p3);
# time to the first pose with the abort kernel in latency mode (abl: groups of
# 2, no exec region for the pivot row) against p4
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
T=r5n AB="p3=lib/libhc_trifocal_p3.so p4=lib/libhc_trifocal_p4.so" bash scripts/gpu_r5f.sh || exit $?
T=r5n BASE=p4 BUILDS=abl bash scripts/gpu_r5j.sh
