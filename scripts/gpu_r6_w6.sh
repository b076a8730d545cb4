# Round 6: the six-wide walk-only tree (RTBVH_W6=1) against the 4-wide one: certified GPU tests under the knob,
# (RTBVH_W6 existed at commit 2b9ee26 only: deleted after this measurement)
# then ROUNDS interleaved ab_trace.py runs (AB_SET=certbase) with the knob off / on
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r06_w6}
if [ -n "${W6_TESTS:-1}" ] && [ "${W6_TESTS:-1}" != 0 ]; then
  RTBVH_W6=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "${W6_K:-certif or auto}" > gpurun_out/${T}_tests.log 2>&1
  rc=$?
  tail -3 gpurun_out/${T}_tests.log
  if [ $rc -ne 0 ]; then echo "W6 TESTS rc=$rc"; grep -E "^(FAILED|E  )" gpurun_out/${T}_tests.log | head -30; exit 1; fi
fi
for r in $(seq 1 ${ROUNDS:-2}); do
  for w in 0 1; do
    out=$(RTBVH_W6=$w AB_COUNTS=${AB_COUNTS:-} AB_SET=certbase AB_ROUNDS=${AB_ROUNDS:-3} timeout -k 10 300 python scripts/ab_trace.py 2>&1) || { echo "$out" | tail -5; exit 1; }
    echo "W6=$w $(echo "$out" | grep -E "ms_med|frame_sha1|internal_visits")" | tee -a gpurun_out/${T}_ab.log
  done
done
echo "call ok"
