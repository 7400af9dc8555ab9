# round 5: the abort kernel's latency-mode LU with consecutive always-live
# column groups stored / read as pairs (lp1; one wait per pair) against v10.2:
# abort-mode parity, then time to the first good pose (config 3)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
T=r5lp BASE=v102 BUILDS="lp1" bash scripts/gpu_r5j.sh
