# round 5: the pivot search narrowed to the candidate rows' quad / half-row /
# row at steps 0..17 with the eligible set carried as a wave mask (sp1), and
# the eligible region narrowed to the candidate rows (sp2), against v10.1
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
bash scripts/gpu_ab.sh r5sp2 v101=lib/libhc_trifocal_v101.so sp1=lib/libhc_trifocal_sp1.so sp2=lib/libhc_trifocal_sp2.so
