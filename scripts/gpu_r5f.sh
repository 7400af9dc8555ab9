# round 5: which part of the scratch-window LU (v3) costs the loaded launch:
# v5 = v3 with the FMAs of each element back to back (v1's order), v6 = v3 with
# the relabel and factor keep after the column groups (v1's placement)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
bash scripts/gpu_ab.sh ${T:-r5f} ${AB:-v1=lib/libhc_trifocal_v1.so v3=lib/libhc_trifocal_v3.so v5=lib/libhc_trifocal_v5.so v6=lib/libhc_trifocal_v6.so}
