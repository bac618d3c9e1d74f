"""Per-kernel sums of a rocprofv3 --pmc pass (its rocpd SQLite output): counter value (KB for
FETCH_SIZE / WRITE_SIZE) and dispatch count per kernel name.
    python tools/pmc_db.py <run_results.db> [name-substring]"""
import collections
import sqlite3
import sys


def per_kernel(db, sub=""):
    c = sqlite3.connect(db)
    q = ("select s.kernel_name, i.name, sum(e.value), count(distinct d.id) from rocpd_pmc_event e "
         "join rocpd_kernel_dispatch d on d.event_id = e.event_id "
         "join rocpd_info_kernel_symbol s on s.id = d.kernel_id join rocpd_info_pmc i on i.id = e.pmc_id "
         "group by s.kernel_name, i.name")
    out = collections.OrderedDict()
    for name, ctr, v, n in c.execute(q):
        if sub in name:
            out[(name, ctr)] = (v, n)
    return out


if __name__ == "__main__":
    for (name, ctr), (v, n) in per_kernel(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "").items():
        print(f"{ctr:12s} {v:14.0f} x{n:<4d} {name[:110]}")
