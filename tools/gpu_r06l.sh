set -o pipefail
cd "${GRAFT_REPO_ROOT}"
bash tools/gpu.sh ab r06l_g16 "WT r6_head" "double" || exit $?
bash tools/gpu.sh ab r06l_g16_48 "WT r6_head" "double" --n-space 3072 --force-variant 1,48 || exit $?
bash tools/gpu.sh tests r06l_tests || exit $?
