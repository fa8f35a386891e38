"""Instruction histogram of one kernel in a hipcc -S listing (device asm).

usage: python tools/asm_hist.py FILE.s NAME_SUBSTRING [--div N] [--top K]
--div divides the counts (e.g. by the rows a kernel body unrolls) to read them per unit of work.
"""
import argparse
import collections
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("name")
    ap.add_argument("--div", type=float, default=1.0)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    s = open(a.asm).read()
    labels = [m for m in re.finditer(r"^(_Z\S+):", s, re.M) if a.name in m.group(1)]
    if not labels:
        raise SystemExit("no kernel matches %r" % a.name)
    m = labels[0]
    body = s[m.end():s.index(".Lfunc_end", m.end())]
    c = collections.Counter()
    for line in body.split("\n"):
        line = line.strip()
        if not line or line.startswith((".", ";", "_")) or line.endswith(":"):
            continue
        c[line.split()[0]] += 1
    d = a.div
    valu = sum(v for k, v in c.items() if k.startswith("v_") and "mfma" not in k)
    mfma = sum(v for k, v in c.items() if "mfma" in k)
    lds = sum(v for k, v in c.items() if k.startswith("ds_"))
    vmem = sum(v for k, v in c.items() if k.startswith(("global_", "buffer_")))
    print("%s\n total %.1f  valu %.1f  mfma %.1f  lds %.1f  vmem %.1f" %
          (m.group(1), sum(c.values()) / d, valu / d, mfma / d, lds / d, vmem / d))
    for k, v in c.most_common(a.top):
        print("%8.1f %s" % (v / d, k))


if __name__ == "__main__":
    main()
