# knobs on the shipped build: SLICE_QBIG 6 / 12 steps (8 shipped), eval look-ahead
# 3 terms (2 shipped); parity of test_gpu_parity.py on ea3, A/B against r4j
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
bash scripts/gpu_ab.sh r4m base=lib/libhc_trifocal_r4j.so qb6=lib/libhc_trifocal_qb6.so qb12=lib/libhc_trifocal_qb12.so ea3=lib/libhc_trifocal_ea3.so
