# rocprofv3 kernel trace of the binned primary pass (C5 frame, AB_SET=binned variants)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out
AB_SET=binned AB_ROUNDS=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_binned -o run -- python3 $R/scripts/ab_trace.py > $R/gpurun_out/prof_binned.log 2>&1 || { echo "PROF FAILED"; tail -20 $R/gpurun_out/prof_binned.log; exit 1; }
cat $R/gpurun_out/prof_binned/run_kernel_stats.csv | cut -d, -f1-8 | head -30
