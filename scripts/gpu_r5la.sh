# round 5: the LU with lookahead (step I+1's pivot search right after the
# column group of step I that holds column I+1): la1 in the abort kernel only
# (time to the first good pose, config 3, after the abort-mode parity tests),
# la2 in the tracking kernel too (config-2 launch A/B + parity) against v10.2
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
T=r5la BASE=v102 BUILDS="la1" bash scripts/gpu_r5j.sh || exit $?
bash scripts/gpu_ab.sh r5la2 v102=lib/libhc_trifocal_v102.so la2=lib/libhc_trifocal_la2.so
