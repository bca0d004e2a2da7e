"""Summarise a rocprofv3 kernel-trace CSV: per kernel name, mean duration; and the mean span of
consecutive kernel runs (launch-to-launch gaps) — for the small-launch study."""
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
dur = collections.defaultdict(list)
for r in rows:
    dur[r["Kernel_Name"].split("(")[0][:70]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in dur.items():
    print(f"{len(v):6d}  {sum(v)/len(v):9.2f} us  {k}")
gaps = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(rows, rows[1:])]
gaps = [g for g in gaps if g < 50]
if gaps:
    gaps.sort()
    print("gap between kernels: median", round(gaps[len(gaps)//2], 2), "us; p10", round(gaps[len(gaps)//10], 2))
