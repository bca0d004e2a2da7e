"""Split a rocprofv3 kernel-trace CSV at idle gaps > 10 ms and print, per segment, each kernel's
mean duration and the mean time per call (segment span / calls of the most frequent kernel)."""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
segs, cur = [], []
for r in rows:
    if cur and int(r["Start_Timestamp"]) - int(cur[-1]["End_Timestamp"]) > 10_000_000:
        segs.append(cur)
        cur = []
    cur.append(r)
segs.append(cur)
for i, s in enumerate(segs):
    dur = collections.defaultdict(list)
    for r in s:
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        dur[name.split("(")[0][:90]].append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    calls = max(len(v) for v in dur.values())
    span = (int(s[-1]["End_Timestamp"]) - int(s[0]["Start_Timestamp"])) / 1e3
    busy = sum(sum(v) for v in dur.values())
    print(f"segment {i}: {calls} calls, {span / calls:.2f} us per call, kernels busy "
          f"{busy / calls:.2f} us per call")
    for k, v in dur.items():
        print(f"   {len(v):6d}  {sum(v) / len(v):9.2f} us  {k}")
