"""Per-dispatch counter values of the last dispatch of kernels matching a substring, over rocprofv3
counter_collection CSVs.  Usage: python tools/pmc_summary.py KERNEL_SUBSTR CSV [CSV ...]"""
import csv
import sys
from collections import defaultdict


def main():
    sub, paths = sys.argv[1], sys.argv[2:]
    for path in paths:
        per = defaultdict(lambda: defaultdict(float))
        for r in csv.DictReader(open(path)):
            if sub in r["Kernel_Name"]:
                per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
        if not per:
            continue
        last = per[max(per)]
        print(path.split("/")[-1], f"({len(per)} dispatches, last shown)")
        for k, v in sorted(last.items()):
            print(f"  {k:32s} {v:.5g}")


if __name__ == "__main__":
    main()
