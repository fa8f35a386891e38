"""Idle gaps between consecutive kernels of a rocprofv3 kernel trace (graph-replayed steps): over the
last N dispatches, span = last end - first start, busy = union of kernel intervals, gaps = span - busy.
Usage: python tools/trace_gaps.py KERNEL_TRACE_CSV [N]"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows)[-n:]
    busy, cur_s, cur_e = 0, None, None
    gaps = []
    for s, e in iv:
        if cur_e is None:
            cur_s, cur_e = s, e
        elif s > cur_e:
            busy += cur_e - cur_s
            gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = iv[-1][1] - iv[0][0]
    small = [g for g in gaps if g < 100000]     # inside a step (< 100 us)
    print(f"{len(iv)} dispatches: span {span / 1e6:.3f} ms, busy {busy / 1e6:.3f} ms, idle {(span - busy) / 1e6:.3f} ms "
          f"({100 * (span - busy) / span:.1f} %); in-step gaps: {len(small)}, mean {sum(small) / max(1, len(small)) / 1e3:.2f} us, "
          f"sum {sum(small) / 1e6:.3f} ms")


if __name__ == "__main__":
    main()
