set -o pipefail
R=$GRAFT_REPO_ROOT
bash $R/profiles/r05/ab.sh r05r config3 3 nip_amd/_lib/ab/widep1.so nip_amd/_lib/ab/widep2.so || exit 1
bash $R/profiles/r05/ab.sh r05r estep_config3 3 nip_amd/_lib/ab/mwp1.so || exit 1
bash $R/profiles/r05/ab.sh r05r fb 2 || exit 1
