set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_pmc.sh build_a4 && bash scripts/gpu_pmc.sh build
