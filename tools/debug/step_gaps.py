"""Per-step composition of the bench's timed loops from a rocprofv3 kernel trace: step length (from one
k_range_dot to the next), kernel busy time, copy/fill kernels, idle. usage: step_gaps.py run_kernel_trace.csv"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "k_range_dot" in r["Kernel_Name"]]
for a, b in zip(starts, starts[1:]):
    seg = rows[a:b]
    t0, t1 = int(seg[0]["Start_Timestamp"]), int(rows[b]["Start_Timestamp"])
    dur = lambda r: int(r["End_Timestamp"]) - int(r["Start_Timestamp"])  # noqa: E731
    busy = sum(dur(r) for r in seg)
    aux = sum(dur(r) for r in seg if "rocclr" in r["Kernel_Name"] or "stage_scatter" in r["Kernel_Name"])
    kind = "dropin" if any("chain_walk" in r["Kernel_Name"] for r in seg) else "index"
    print("%-6s step %7.3f ms  compute %7.3f  copies %.3f  idle %.3f  kernels %d"
          % (kind, (t1 - t0) / 1e6, (busy - aux) / 1e6, aux / 1e6, (t1 - t0 - busy) / 1e6, len(seg)))
