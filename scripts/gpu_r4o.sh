# parity of the fuse variant (one column-group test per group and step: the
# pivot lanes store the group and the rows below update it in the same branch)
# on test_gpu_parity.py, then its A/B against the shipped build (r4j)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
bash scripts/gpu_ab.sh r4o base=lib/libhc_trifocal_r4j.so fuse=lib/libhc_trifocal_fuse.so
