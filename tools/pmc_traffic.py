"""HBM traffic per launch from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; one counter group per
pass, MI355X_MICROARCH.md 'HBM'): bytes = 2 x FETCH_SIZE x 1024 (gfx950 FETCH_SIZE counts half the
bytes of a wide streaming read) + WRITE_SIZE x 1024, averaged over every dispatch of a kernel.
Writes {workload: {kernel: {...}}} into a JSON file that bench.py reads for roofline.traffic.

Usage: python tools/pmc_traffic.py FETCH_CSV WRITE_CSV OUT_JSON WORKLOAD [GRAPH_STEPS]
GRAPH_STEPS: keep only the dispatches of the last GRAPH_STEPS replayed graph steps (graph_step_census.py run)."""
import csv
import json
import os
import re
import sys
from collections import defaultdict


_DEMANGLED = {}


def demangle(name):
    """Itanium-mangled kernel symbol -> C++ name (c++filt); unchanged when it is not mangled."""
    if not name.startswith("_Z"):
        return name
    if name not in _DEMANGLED:
        import subprocess
        try:
            # binutils' c++filt predates the _Float16 / __bf16 manglings: spell them as half / a vendor type
            m = name.replace("DF16_", "Dh").replace("DF16b", "u6__bf16")
            out = subprocess.run(["c++filt", m], capture_output=True, text=True).stdout.strip()
            _DEMANGLED[name] = out.replace("half", "_Float16") if out and out != m else name
        except OSError:
            _DEMANGLED[name] = name
    return _DEMANGLED[name]


def kernel_key(name):
    """rocprofv3 kernel name -> the instantiation name bench.py reports (svk_last_kernel form)."""
    n = demangle(name.strip())
    if n.startswith("void "):
        n = n[5:]
    n = n.replace("svk::", "")
    depth = 0
    for i, ch in enumerate(n):      # cut the argument list: first '(' outside template brackets
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            return _family(n[:i])
    return _family(n)


def _family(n):
    """gemm_pk's PERM template argument (round 6: the same kernel with the W rows permuted so the epilogue operands
    load as 16-byte pieces) is not part of the instantiation name bench.py reports: both variants are one family."""
    if n.startswith("gemm_pk<") and n.count(",") >= 11:
        for tail in (", true>", ", false>"):
            if n.endswith(tail) and n[: -len(tail)].count(",") >= 10:
                return n[: -len(tail)] + ">"
    return n


def graph_step_dispatches(path, steps, last_kernel="mean_rows"):
    """Dispatch ids of the last ``steps`` replayed graph steps of a counter CSV (the counter
    passes must describe the product step only).  The profiled program (tools/graph_step_census.py run) ends
    with ``steps`` replays of the captured extraction step and nothing else; dispatches are ordered by id and
    split after each step's last kernel (``last_kernel``).  Returns (ids, per-step launch counts)."""
    order = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            d = int(r.get("Dispatch_Id") or r.get("Correlation_Id"))
            order[d] = r["Kernel_Name"]
    groups, cur = [], []
    for d in sorted(order):
        cur.append(d)
        if last_kernel in order[d]:
            groups.append(cur)
            cur = []
    use = groups[-steps:]
    if len(use) < steps:
        raise SystemExit(f"{path}: only {len(use)} complete steps found, {steps} asked")
    return {d for g in use for d in g}, [len(g) for g in use]


def per_kernel(path, counter, keep=None):
    vals = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            if keep is not None and int(r.get("Dispatch_Id") or r.get("Correlation_Id")) not in keep:
                continue
            if r["Counter_Name"] == counter:
                vals[kernel_key(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return vals


def main():
    fetch_csv, write_csv, out_json, workload = sys.argv[1:5]
    gsteps = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    kf = graph_step_dispatches(fetch_csv, gsteps)[0] if gsteps else None
    kw = graph_step_dispatches(write_csv, gsteps)[0] if gsteps else None
    fetch, write = per_kernel(fetch_csv, "FETCH_SIZE", kf), per_kernel(write_csv, "WRITE_SIZE", kw)
    table = {}
    for k in sorted(set(fetch) & set(write)):
        f, w = fetch[k], write[k]
        fk, wk = sum(f) / len(f), sum(w) / len(w)
        table[k] = {"dispatches": len(f), "fetch_size_kb_avg": round(fk, 1), "write_size_kb_avg": round(wk, 1),
                    "hbm_bytes_per_launch": round((2.0 * fk + wk) * 1024.0)}
    data = {}
    if os.path.exists(out_json):
        with open(out_json) as fh:
            data = json.load(fh)
    data[workload] = {"source": [os.path.relpath(fetch_csv), os.path.relpath(write_csv)],
                      "scope": (f"the last {gsteps} graph-replayed steps only" if gsteps else "every dispatch"),
                      "formula": "(2 * FETCH_SIZE + WRITE_SIZE) * 1024 per dispatch, averaged", "kernels": table}
    with open(out_json, "w") as fh:
        json.dump(data, fh, indent=1, sort_keys=True)
    for k, v in sorted(table.items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"] * kv[1]["dispatches"])[:15]:
        print(f"{v['hbm_bytes_per_launch'] / 1e6:10.2f} MB/launch  n={v['dispatches']:5d}  {k[:110]}")


if __name__ == "__main__":
    main()
