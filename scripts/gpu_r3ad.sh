# rare-test A/B (scripts/gpu_r3ac.sh), then the full round-3 validation of HEAD (scripts/gpu_r3ab.sh)
cd $GRAFT_REPO_ROOT
bash scripts/gpu_r3ac.sh && bash scripts/gpu_r3ab.sh
