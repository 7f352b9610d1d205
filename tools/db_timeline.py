"""Step timeline from a rocprofv3 rocpd database (the default output format):
python tools/db_timeline.py RESULTS.db NAME_SUBSTR INDEX [SKIP_SUBSTR]
Prints every dispatch from the INDEX-th launch of NAME_SUBSTR to the next one, times in
us from its start, leaving out names containing SKIP_SUBSTR (default k_st_: the window)."""
import sqlite3
import sys

path, key, k = sys.argv[1], sys.argv[2], int(sys.argv[3])
skip = sys.argv[4] if len(sys.argv) > 4 else "k_st_"
r = list(sqlite3.connect(path).execute(
    "select start, end, stream_id, queue_id, name from kernels order by start"))
idx = [i for i, x in enumerate(r) if key in x[4]]
i, j = idx[k], idx[k + 1]
t0 = r[i][0]
nskip = 0
for s, e, st, q, name in r[i - 6:j + 1]:
    if skip and skip in name:
        nskip += 1
        continue
    print(f"{(s - t0) / 1000:9.2f} {(e - t0) / 1000:9.2f} dur {(e - s) / 1000:7.2f}  s{st} q{q} {name[:70]}")
print(f"step length {(r[j][0] - t0) / 1000:.1f} us; {nskip} window dispatches not listed")
