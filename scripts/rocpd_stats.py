"""Per-kernel table (calls, average / total us) from a rocprofv3 rocpd database (the default
output of this ROCm's rocprofv3 when --output-format is not csv):
python scripts/rocpd_stats.py <results.db> [n]"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name = "kernel_name" if "kernel_name" in cols else "name"
q = (f"select {name}, count(*), avg(end - start), sum(end - start) from kernels "
     f"group by {name} order by sum(end - start) desc limit {n}")
for k, calls, avg, tot in c.execute(q):
    print(f"{k[:78]:78s} {calls:6d} {avg / 1e3:9.1f} us  {tot / 1e6:8.3f} ms")
