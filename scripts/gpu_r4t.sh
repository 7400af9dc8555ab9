# column groups of 4 with the fused group test in the tracking kernels (fuse4)
# against the shipped build (groups of 2, fused); parity on fuse4
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
bash scripts/gpu_ab.sh r4t base=lib/libhc_trifocal_r4r.so fuse4=lib/libhc_trifocal_fuse4.so
