# the shipped build's trace + PMC with 30 timed launches (the process's cold
# first launch weighs 1/34 in the rocprof average), then the N=2 rehearsal
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
bash scripts/profile.sh r4l || exit 1
bash scripts/gpu_r4_n2.sh r4l
