# round 5: GPU tests of the product build, the bare `bench.py --gpus 2`
# rehearsal, then the A/B of the eligible-rows LU groups (v1: pivot lane to the
# buffer, v2: scratch windows) against it
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
bash scripts/gpu_r5a.sh r5b || exit $?
bash scripts/gpu_ab.sh r5b base=lib/libhc_trifocal_r5base.so v1=lib/libhc_trifocal_v1.so v2=lib/libhc_trifocal_v2.so
