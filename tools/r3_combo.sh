# Round-3: A/B 7 then the extra evidence (forecast, tiny sizes, SQ, rehearsal).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/r3_ab7.sh || exit $?
bash tools/r3_extra.sh sf1 sq1
