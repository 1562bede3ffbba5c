"""Print the kernels of the last replayed step in a rocprofv3 kernel trace: duration and the gap
before each (usage: python tools/last_step.py gpurun_out/trace_c2/run_kernel_trace.csv [n])."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
prev = None
for r in rows[-n:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1000 if prev else 0.0
    print(f"{(e - s) / 1000:8.1f} us  gap {gap:7.1f}  q{r.get('Queue_Id', '?'):>3}  {r['Kernel_Name'][:100]}")
    prev = max(prev or 0, e)
