# Round 6 A/B of library builds in one GPU call: ROUNDS x libs interleaved, AB_SET (default certbase) mode,
# ab_trace.py's median ms and stage times per library
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
ROUNDS=${ROUNDS:-2} AB_SET=${AB_SET:-certbase} AB_ROUNDS=${AB_ROUNDS:-3} bash scripts/ab_libs.sh "$@"
