"""Kernel summary from a rocprofv3 rocpd database: name, calls, avg us, total ms."""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
q = ("select substr(name,1,110), count(*), avg(duration)/1000.0, sum(duration)/1e6 from kernels "
     "group by name order by sum(duration) desc limit 15")
for r in c.execute(q):
    print(f"{r[3]:10.3f} ms {r[1]:6d} x {r[2]:10.2f} us  {r[0]}")
