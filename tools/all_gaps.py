"""Every idle gap > 25 us in a rocprofv3 kernel trace with its neighbours: python tools/all_gaps.py TRACE.csv"""
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
def sh(n): return n.replace("void ","").replace("at::native::","").replace("mx::","").split("(")[0][:50]
end=0
for i,r in enumerate(rows):
    s,e=int(r["Start_Timestamp"]),int(r["End_Timestamp"])
    gap=(s-end)/1000
    if gap>25 and i>0:
        print(f"{gap:7.1f} us before {sh(r['Kernel_Name']):50s} after {sh(rows[i-1]['Kernel_Name'])}")
    end=max(end,e)
