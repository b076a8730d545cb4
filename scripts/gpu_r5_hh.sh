# Round 5, call hh: the bounce walk's persistent grid for a rank's shard at N = 8 / 4 (RTBVH_BOUNCE_BLOCKS;
# default 1024 below 4M pixels), four frames in flight and one frame at a time, two rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r05_hh}
for rnd in 1 2; do
for B in 512 768 1024 1536 2048; do
  for NR in "8 1" "4 1"; do
    set -- $NR
    RTBVH_BOUNCE_BLOCKS=$B timeout -k 10 300 python3 scripts/rank_prof.py $1 $2 40 inflight 4 > gpurun_out/${T}_b${B}_n$1_inflight_$rnd.json 2>> gpurun_out/${T}.err || { tail -5 gpurun_out/${T}.err; exit 1; }
    RTBVH_BOUNCE_BLOCKS=$B timeout -k 10 300 python3 scripts/rank_prof.py $1 $2 20 > gpurun_out/${T}_b${B}_n$1_one_$rnd.json 2>> gpurun_out/${T}.err || { tail -5 gpurun_out/${T}.err; exit 1; }
    echo "r$rnd B$B N$1 inflight $(grep -o '"ms_per_frame_host": [0-9.]*' gpurun_out/${T}_b${B}_n$1_inflight_$rnd.json) one $(grep -o '"ms_per_frame_host": [0-9.]*' gpurun_out/${T}_b${B}_n$1_one_$rnd.json)"
  done
done
done
echo "call ok"
