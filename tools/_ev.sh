set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_profile_all.sh r01b double && bash tools/pmc_traffic.sh r01b double
