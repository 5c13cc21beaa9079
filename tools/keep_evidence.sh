#!/bin/bash
# Copy a tools/gpu_final.sh run (gpurun_out/$1) into profiles/$2 (tracked): logs, PMC records,
# rocprofv3 kernel stats (the PMC records are already in profiles/$ROUND, where bench.py reads them).
set -e
S=gpurun_out/$1; D=profiles/$2
mkdir -p $D
cp $S/*.log $S/pmc_*.json $D/
cp $S/prof/prof_kernel_stats.csv $D/kernel_stats_stance_cold_b4096.csv
for c in rl_random_b8192 modes16_b16384; do cp $S/prof_$c/prof_kernel_stats.csv $D/kernel_stats_$c.csv; done

