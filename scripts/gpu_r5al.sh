# round 5: four more column groups run without a test (al90: the groups live
# in >= 90 % of the sampled solves, profiles/r5lv_live.jsonl) against v10.2
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
bash scripts/gpu_ab.sh r5al v102=lib/libhc_trifocal_v102.so al90=lib/libhc_trifocal_al90.so
