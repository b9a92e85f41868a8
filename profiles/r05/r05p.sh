set -o pipefail
R=$GRAFT_REPO_ROOT
bash $R/profiles/collect.sh r05p config3 em estep_config3 || exit 1
echo collected
