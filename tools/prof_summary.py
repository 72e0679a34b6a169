"""Print the rocprofv3 kernel stats + one pass of the kernel trace (tools helper)."""
import signal

signal.signal(signal.SIGPIPE, signal.SIG_DFL)
import csv
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
rows = list(csv.DictReader(open(f"{d}/bench_kernel_stats.csv")))
for r in rows:
    print(r["Name"][:50].ljust(50), r["Calls"].rjust(5), "%8.2f us avg" % (float(r["AverageNs"]) / 1e3),
          "%5.1f%%" % float(r["Percentage"]))
tr = list(csv.DictReader(open(f"{d}/bench_kernel_trace.csv")))
tr.sort(key=lambda r: int(r["Start_Timestamp"]))
seq = tr[-40:]
t0 = int(seq[0]["Start_Timestamp"])
print("--- tail of trace: start(us) dur(us) grid wg vgpr lds")
for r in seq[:14]:
    print(r["Kernel_Name"][:34].ljust(34), "%8.2f %7.2f" % ((int(r["Start_Timestamp"]) - t0) / 1e3,
          (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3), r["Grid_Size_X"], r["Workgroup_Size_X"],
          r["VGPR_Count"], r["LDS_Block_Size"])
