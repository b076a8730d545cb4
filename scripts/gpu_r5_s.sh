# Round 5, call s: frames in flight per rank, 4 / 6 / 8 (a library with 8 buffer sets), in the certified mode at
# N = 1 and the N = 8 deal (scripts/rank_sim_cert.py: every rank's bands on this one GPU).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r05_s}
for F in 4 6 8; do
  RTBVH_LIB=$(realpath ablib/librtbvh_ms8.so) timeout -k 10 600 python scripts/rank_sim_cert.py 20 $F 1,8 > gpurun_out/${T}_F$F.json 2> gpurun_out/${T}_F$F.err || { echo "RANK SIM F=$F FAILED"; tail -5 gpurun_out/${T}_F$F.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], {k:(v['max_ms_in_flight'], v['max_ms_one_frame'], v.get('speedup_compute_only_in_flight')) for k,v in d.items()})" gpurun_out/${T}_F$F.json F$F
done
echo "call ok"
