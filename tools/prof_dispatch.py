"""Per-dispatch kernel durations from a rocprofv3 --kernel-trace results database (tool)."""
import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
rows = list(c.execute("select name, start, end, grid_x from kernels order by start"))
skip = int(sys.argv[2]) if len(sys.argv) > 2 else 0
for nm, s, e, g in rows[skip:]:
    print(f"{nm.split('(')[0][-34:]:36s} {(e - s) / 1000:10.1f} us  grid {g}")
