#!/bin/bash
# Copy the judged outputs of scripts/gpu_round.sh from gpurun_out/ into profiles/ under a tag:
#   scripts/save_profiles.sh r02_s4b
set -e
T=${1:?tag}
cd "$(dirname "$0")/.."
cp gpurun_out/bench.json profiles/${T}_bench.json
cp gpurun_out/gpu_tests.log profiles/${T}_gpu_tests.log
cp gpurun_out/prof_bench/run_kernel_stats.csv profiles/${T}_kernel_stats.csv
python3 scripts/trace_summary.py gpurun_out/prof_bench/run_kernel_trace.csv profiles/${T}_kernel_trace_summary.json
cp gpurun_out/counts_round.json profiles/${T}_counts_c5_nearest-first-wide.json
# the PMC the box's bench read (gpu_round.sh copied it into the box's profiles/, which does not come back)
cp gpurun_out/pmc_c5_round.json profiles/pmc_c5_${PMC_NAME:-nearest-first-wide-binned}.json
ls -la profiles/${T}_*
