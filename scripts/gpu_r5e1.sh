# round 5: the eligible-rows mask carried from step to step (el1: elig_{I+1} =
# elig_I && !is_piv_I, no rowid compare) against the shipped build (base6)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
bash scripts/gpu_ab.sh r5e1 base6=lib/libhc_trifocal_base6.so el1=lib/libhc_trifocal_el1.so
