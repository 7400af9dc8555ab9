# parity of the tie4 variant (inline tie resolution at pivot steps 18, 19, 21,
# 22) on test_gpu_parity.py, then an A/B of the round-3 product (r4c), the
# current sources (r4f: prefix places by LDS bank, inline ties at 18 and 21,
# reciprocal factors in their own pairs, no f64 division in the RK weight) and tie4
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
bash scripts/gpu_ab.sh r4f base=lib/libhc_trifocal_r4c.so r4f=lib/libhc_trifocal_r4f.so tie4=lib/libhc_trifocal_tie4.so
