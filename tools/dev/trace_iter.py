"""Average per-launch durations of one GN iteration in a rocprofv3 kernel trace: the iteration's launches in start order,
between consecutive launches of an anchor kernel, averaged position by position over the last iterations.
   python tools/dev/trace_iter.py gpurun_out/prof_C5/run_kernel_trace.csv [anchor] [iterations]"""
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
anchor = sys.argv[2] if len(sys.argv) > 2 else "k_warp_mesh_quad"
n_it = int(sys.argv[3]) if len(sys.argv) > 3 else 50
seq = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:48]) for r in rows))
idx = [i for i, s in enumerate(seq) if anchor in s[2]]
its = [seq[idx[j]:idx[j + 1]] for j in range(max(0, len(idx) - n_it - 5), len(idx) - 5)]
L = min(len(it) for it in its)
its = [it for it in its if len(it) == L]
tot = 0.0
for p in range(L):
    d = statistics.mean((it[p][1] - it[p][0]) / 1000 for it in its)
    gap = statistics.mean((it[p][0] - it[p - 1][1]) / 1000 for it in its) if p else 0.0
    tot += d
    print(f"{p:2d} {its[0][p][2]:48s} {d:7.2f} us  (gap before {gap:5.2f})")
span = statistics.mean((it[-1][1] - it[0][0]) / 1000 for it in its)
print(f"sum of launches {tot:.1f} us, first start -> last end {span:.1f} us over {len(its)} iterations")
