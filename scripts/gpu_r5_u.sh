# Round 5, call u: frames in flight x hardware queues at N = 4 and N = 8 (rank_sim_cert, certified, every
# rank's bands on this one GPU; a library with 8 buffer sets): (F, GPU_MAX_HW_QUEUES) = (4, 4), (8, 8), (6, 8).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r05_u}
for cfg in 4:4 8:8 6:8 4:4; do
  F=${cfg%%:*}; Q=${cfg##*:}
  GPU_MAX_HW_QUEUES=$Q RTBVH_LIB=$(realpath ablib/librtbvh_ms8.so) timeout -k 10 600 python scripts/rank_sim_cert.py 20 $F 4,8 > gpurun_out/${T}_F${F}_Q${Q}.json 2> gpurun_out/${T}_F${F}_Q${Q}.err || { echo "RANK SIM FAILED"; tail -5 gpurun_out/${T}_F${F}_Q${Q}.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], {k:(v['max_ms_in_flight'], v['max_ms_one_frame']) for k,v in d.items()})" gpurun_out/${T}_F${F}_Q${Q}.json F${F}_Q${Q}
done
echo "call ok"
