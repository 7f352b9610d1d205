# r05ab: the reservoir's CU count beside SPEEDY's 64 (SML_RES_CUS), same box
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu/ab_bench.sh r05ab "SML_RES_CUS=192" "SML_RES_CUS=176" "SML_RES_CUS=160"
