"""Summarise rocprofv3 --pmc sqlite outputs (rocpd *.db): mean counter value per dispatch of the kernels
whose name contains a pattern.   python tools/pmc_db.py PATTERN DB [DB ...]"""
import collections
import sqlite3
import sys


def main():
    pat, dbs = sys.argv[1], sys.argv[2:]
    for db in dbs:
        c = sqlite3.connect(db)
        kn = {e: (n, st, en) for e, n, st, en in c.execute(
            "select d.event_id, s.kernel_name, d.start, d.end from rocpd_kernel_dispatch d "
            "join rocpd_info_kernel_symbol s on d.kernel_id = s.id")}
        agg = collections.defaultdict(dict)
        for ev, name, val in c.execute("select e.event_id, i.name, e.value from rocpd_pmc_event e "
                                       "join rocpd_info_pmc i on e.pmc_id = i.id"):
            if pat in kn.get(ev, ("",))[0]:
                agg[name][ev] = agg[name].get(ev, 0.0) + val
        durs = sorted((en - st) / 1000 for (n, st, en) in kn.values() if pat in n)
        print(f"{db}: {len(durs)} dispatches, median {durs[len(durs) // 2] if durs else 0:.1f} us")
        for name in sorted(agg):
            v = list(agg[name].values())
            print(f"  {name:28s} {sum(v) / len(v):16.0f}")


if __name__ == "__main__":
    main()
