# parity of the current sources (w6c: RK weights without f64 division, parallel
# prefix collection, bank-aware prefix places) on test_gpu_parity.py, A/B of the round-4 trims against the
# product, then the N=2 bench rehearsal (two ranks on cuda:0 over gloo)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
bash scripts/gpu_ab.sh r4e base=lib/libhc_trifocal_r4c.so w6rcp=lib/libhc_trifocal_w6rcp.so w6tie=lib/libhc_trifocal_w6tie.so w6h=lib/libhc_trifocal_w6h.so w6c=lib/libhc_trifocal_w6c.so || exit 1
bash scripts/gpu_r4_n2.sh r4e
