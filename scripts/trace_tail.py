"""Print the last N gw:: kernels of a rocprofv3 kernel trace with durations (us)."""
import csv
import sys

path = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows = [r for r in csv.DictReader(open(path)) if "gw::" in r["Kernel_Name"]]
for r in rows[-n:]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
    print(f"{r['Kernel_Name'][:44]:44s} {d:9.1f} us  grid={r['Grid_Size_X']} lds={r['LDS_Block_Size']} vgpr={r['VGPR_Count']}")
