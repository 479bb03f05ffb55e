"""Per-kernel count / average / total duration (us) from a rocprofv3 results database
(design tool): python3 tools/kstats.py gpurun_out/<dir>/run_results.db"""
import sqlite3
import sys

for path in sys.argv[1:]:
    c = sqlite3.connect(path)
    print(path)
    for name, n, avg, tot in c.execute(
            "select name, count(*), avg(duration)/1000.0, sum(duration)/1000.0 from kernels group by name order by 4 desc"):
        print("  %-40s %5d  avg %10.1f us  total %10.1f us" % (name.split("(")[0], n, avg, tot))
