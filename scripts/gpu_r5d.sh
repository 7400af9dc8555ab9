# round 5: A/B of the scratch-window LU groups with fresh lane ids in park /
# update (v3) against the round-4 LU (base) and the eligible-rows groups (v1)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
bash scripts/gpu_ab.sh ${T:-r5d} base=lib/libhc_trifocal_r5base.so v1=lib/libhc_trifocal_v1.so v3=lib/libhc_trifocal_v3.so v4=lib/libhc_trifocal_v4.so
