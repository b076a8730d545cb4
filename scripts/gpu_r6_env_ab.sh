# Round 6: A/B of env knobs on one library (ab_trace.py AB_SET=certbase), ROUNDS interleaved; VARIANTS ';'-separated
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
IFS=';' read -ra VS <<< "${VARIANTS:?}"
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in "${VS[@]}"; do
    out=$(env $v AB_SET=certbase AB_ROUNDS=${AB_ROUNDS:-3} timeout -k 10 300 python scripts/ab_trace.py 2>&1) || { echo "$out" | tail -5; exit 1; }
    echo "$v $(echo "$out" | grep -E "ms_med|frame_sha1" | tr '\n' ' ')"
  done
done
echo "call ok"
