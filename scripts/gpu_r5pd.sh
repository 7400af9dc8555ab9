# round 5: abort-mode issue priority levels by finer queue fractions (pd32:
# the first 1/32 of a launch's paths at 3, the next at 2, ...; pd64: 1/64)
# against v10.2 (1/16): time to the first good pose, config 3
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
T=r5pd BASE=v102 BUILDS="pd32 pd64" bash scripts/gpu_r5j.sh
