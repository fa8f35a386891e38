"""Summarise a rocprofv3 ``--kernel-trace --stats --output-format csv`` kernel_stats.csv into
per-step kernel times.  Usage: python tools/prof_stats.py run_kernel_stats.csv STEPS [TOP]
STEPS = a number, or auto:NAME_SUBSTR: the call count of the (first) kernel whose name contains
NAME_SUBSTR and which runs exactly once per step (e.g. mean_rows_kernel for extraction, sgd for training)."""
import csv
import sys


def main():
    path, steps_arg = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    with open(path) as f:
        rows = list(csv.DictReader(f))
    if steps_arg.startswith("auto:"):
        sub = steps_arg[5:]
        steps = float(next(int(r["Calls"]) for r in rows if sub in r["Name"]))
    else:
        steps = float(steps_arg)
    tot = sum(float(r["TotalDurationNs"]) for r in rows) / 1e6
    print(f"total kernel time {tot / steps:.3f} ms per step ({steps:g} steps; rocprofv3 kernel_stats)")
    for r in rows[:top]:
        ms = float(r["TotalDurationNs"]) / 1e6
        print(f"{ms / steps:8.3f} ms/step  n/step={int(r['Calls']) / steps:6.1f}  avg={float(r['AverageNs']) / 1e3:8.1f}us  "
              f"{float(r['Percentage']):5.2f}%  {r['Name'][:130]}")


if __name__ == "__main__":
    main()
