"""Print a kernel timeline from a rocprofv3 kernel_trace.csv around the N-th launch
of a kernel: python tools/trace_timeline.py TRACE.csv NAME_SUBSTR INDEX [BEFORE AFTER]"""
import csv
import sys

path, key, k = sys.argv[1], sys.argv[2], int(sys.argv[3])
before = int(sys.argv[4]) if len(sys.argv) > 4 else 10
after = int(sys.argv[5]) if len(sys.argv) > 5 else 40
r = sorted(csv.DictReader(open(path)), key=lambda x: int(x["Start_Timestamp"]))
idx = [i for i, x in enumerate(r) if key in x["Kernel_Name"]]
i = idx[k]
t0 = int(r[i]["Start_Timestamp"])
for x in r[max(0, i - before):i + after]:
    print(f"{(int(x['Start_Timestamp']) - t0) / 1000:9.1f} {(int(x['End_Timestamp']) - t0) / 1000:9.1f} "
          f"q{x['Queue_Id']} s{x['Stream_Id']} {x['Kernel_Name'][:60]}")
