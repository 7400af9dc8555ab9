# parity of the rng variant (deferred fast-reciprocal range check: the common
# pivot paths keep the min / max pivot key, one ballot after the forward pass
# sends an out-of-range solve to the dense re-solve) on test_gpu_parity.py,
# then an A/B against the round-4 product (r4g)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
bash scripts/gpu_ab.sh r4h base=lib/libhc_trifocal_r4g.so rng=lib/libhc_trifocal_rng.so
