"""dev/pmcdb.py DIR... -- per-kernel average of every PMC counter in rocprofv3 result DBs."""
import glob
import sqlite3
import sys
from collections import defaultdict

for d in sys.argv[1:]:
    for db in glob.glob(f"{d}/*.db"):
        con = sqlite3.connect(db)
        q = """select s.display_name, k.id, p.name, e.value, k.end - k.start
               from rocpd_pmc_event e join rocpd_kernel_dispatch k on e.event_id = k.event_id
               join rocpd_info_pmc p on e.pmc_id = p.id
               join rocpd_info_kernel_symbol s on k.kernel_id = s.id"""
        agg = defaultdict(lambda: defaultdict(list))
        dur = defaultdict(dict)
        for name, kid, cname, val, ns in con.execute(q):
            agg[name][cname].append(val)
            dur[name][kid] = ns
        print(f"== {db}")
        for name, cs in agg.items():
            n = len(dur[name])
            print(f"  {name[:110]}  launches={n} avg_ms={sum(dur[name].values()) / n / 1e6:.3f}")
            for c, vs in sorted(cs.items()):
                print(f"      {c:40s} {sum(vs) / n:16.4g}")
