#!/bin/bash
# copy a round-6 measurement pass (gpurun_out/$TAG from tools/dev/final_r06.sh) into profiles/r06_*
set -eu
TAG=${TAG:-r06f}
S=gpurun_out/$TAG
for c in C2 C3 C5; do
	lc=$(echo $c | tr 'A-Z' 'a-z')
	cp $S/pmc_traffic_$c.json profiles/r06_pmc_traffic_$lc.json
	cp "$(find $S/prof_$c -name '*kernel_stats.csv' | head -1)" profiles/r06_bench_kernel_stats_$lc.csv
done
cp $S/sq_summary_C2.txt profiles/r06_sq_summary_c2.txt
cp $S/line_c2.json profiles/r06_bench_line.json
for l in c1 c1_arap c2_arap_frame c3 c5 replicas8; do cp $S/line_$l.json profiles/r06_bench_line_$l.json; done
tail -1 $S/smoke.log > profiles/r06_smoke.txt
ls -la profiles/r06_*
