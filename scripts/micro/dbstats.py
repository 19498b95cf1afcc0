"""Per-kernel duration summary (by name and grid) from a rocprofv3 results.db."""
import sqlite3
import sys

for f in sys.argv[1:]:
    c = sqlite3.connect(f)
    print("==", f)
    q = ("select substr(name,1,60), grid_x, grid_y, grid_z, count(*), avg(duration)/1000.0, "
         "min(duration)/1000.0 from kernels group by name, grid_x, grid_y, grid_z order by min(id)")
    for r in c.execute(q):
        print("%-60s %7d %3d %3d n=%3d avg %8.2f us min %8.2f" % r)
