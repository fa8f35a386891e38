"""Where the runtime's copy / fill kernels sit in the train step (37 __amd_rocclr_copyBuffer and
18 __amd_rocclr_fillBufferAligned launches per step).  Run under rocprofv3 --kernel-trace:
  rocprofv3 --kernel-trace --output-format csv -d D -o run -- python bench.py --workload train --no-graph ...
then: python tools/train_copy_census.py D/.../run_kernel_trace.csv
Splits the trace into steps at the SGD kernel, takes the last complete step and prints every runtime kernel
with its neighbours (the svk kernels on either side locate the torch op in svk/train.py)."""
import collections
import csv
import sys


def short(n):
    return n.replace("_ZN3svk", "svk::")[:80]


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    steps, cur = [], []
    for r in rows:
        cur.append(r)
        if "sgd_kernel" in r["Kernel_Name"]:
            steps.append(cur)
            cur = []
    st = steps[-1]
    names = [r["Kernel_Name"] for r in st]
    cnt = collections.Counter(n for n in names if n.startswith("__amd"))
    print(f"{len(steps)} steps; last: {len(st)} launches, runtime kernels {dict(cnt)}")
    for i, n in enumerate(names):
        if n.startswith("__amd"):
            d = (int(st[i]["End_Timestamp"]) - int(st[i]["Start_Timestamp"])) / 1e3
            ctx = " | ".join(short(x) for x in names[max(0, i - 2):i])
            nxt = " | ".join(short(x) for x in names[i + 1:i + 3])
            print(f"#{i:4d} {n[:28]:28s} {d:6.1f} us   after: {ctx}   before: {nxt}")


if __name__ == "__main__":
    main()
