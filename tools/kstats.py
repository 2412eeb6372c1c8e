import sqlite3, sys, numpy as np
c = sqlite3.connect(sys.argv[1])
q = """select name, count(*), avg(end-start), min(end-start), sum(end-start) from kernels group by name order by sum(end-start) desc limit 14"""
for r in c.execute(q): print(f"{r[0][:70]:70s} n={r[1]:6d} avg={r[2]/1e3:9.2f}us min={r[3]/1e3:8.2f}us tot={r[4]/1e6:8.2f}ms")
