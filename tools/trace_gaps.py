"""Print the kernels of the last complete render call of a rocprofv3 kernel trace (calls start at
k_frame_dyn) with durations and the gaps between them."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "k_frame_dyn" in r["Kernel_Name"]]
a, b = idx[-2], idx[-1]
prev, tot = None, 0.0
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1000 if prev else 0.0
    tot += (e - s) / 1000
    print(f"{r['Kernel_Name'][:40]:40s} dur={(e - s) / 1000:8.1f} gap={gap:6.1f} grid={r['Grid_Size_X']} "
          f"lds={r['LDS_Block_Size']} vgpr={r['VGPR_Count']} scr={r['Scratch_Size']}")
    prev = e
print(f"kernel time {tot:.1f} us, span {(int(rows[b - 1]['End_Timestamp']) - int(rows[a]['Start_Timestamp'])) / 1000:.1f} us")
