# rocprofv3 kernel trace of one rank's share of the C5 frame (scripts/rank_prof.py N RANK K: certified walks, the
# bench's band deal, one frame at a time), summarised per frame by scripts/frame_timeline.py (split at k_zero) into
# gpurun_out/${TAG}_rank_timeline_n${N}_r${RANK}.json.  Env: TAG, N (8), RANK (7), K (30)
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r06_rt}; N=${N:-8}; RANK=${RANK:-7}; K=${K:-30}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_prof -o run -- python3 $R/scripts/rank_prof.py $N $RANK $K > $R/gpurun_out/${TAG}_rank_prof.log 2>&1 || { echo "PROF FAILED"; tail -5 $R/gpurun_out/${TAG}_rank_prof.log; exit 1; }
python3 $R/scripts/frame_timeline.py $R/gpurun_out/${TAG}_prof/run_kernel_trace.csv $R/gpurun_out/${TAG}_rank_timeline_n${N}_r${RANK}.json k_zero
