"""Per-grid diff_head timing from a rocprofv3 database: python tools/head_stats.py gpurun_out/hprof/run_results.db"""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
q = "select grid_x/512, count(*), avg(duration)/1000.0 from kernels where name like '%diff_head%' group by grid_x order by grid_x desc limit 5"
for g, n, us in db.execute(q):
    M = g * 128
    fl = 2 * M * 384 * 1152 + 2 * M * 100 * 1152
    print(f"tiles {g} launches {n} {us:.1f} us {fl / us / 1e6:.1f} TFLOP/s")
