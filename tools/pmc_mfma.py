"""MFMA busy fraction from one rocprofv3 counter pass (``--pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
SQ_BUSY_CU_CYCLES``; one SQ group + one GRBM counter fit one pass).

Per dispatch: kernel cycles = GRBM_GUI_ACTIVE / 8 (rocprofv3 sums it over the 8 XCDs,
MI355X_MICROARCH.md 'DVFS give-back'); MFMA busy fraction = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x
kernel cycles).  Whole step = sums over every dispatch of the profiled steps (kernel-active time only;
inter-kernel gaps are not counted).  ``calibration`` = measured MFMA busy cycles of the dominant GEMM /
its algorithmic MFMA cycles (FLOPs / 1024: a v_mfma_f32_16x16x32 instruction is 16384 FLOP in 16
cycles), i.e. how the counter's unit relates to issued MFMA work on this ROCm.

Usage: python tools/pmc_mfma.py COUNTER_CSV OUT_JSON KEY STEPS [KERNEL_SUBSTR FLOP_PER_LAUNCH] [--graph]
--graph: STEPS is the number of graph replays the profiled program ended with (tools/graph_step_census.py run);
only those dispatches are counted (the product step: no eager warm-up, input staging or torch copies), and the
per-step figures divide by that true number of steps."""
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import graph_step_dispatches, kernel_key   # noqa: E402


def main():
    argv = [a for a in sys.argv[1:] if a != "--graph"]
    graph = "--graph" in sys.argv
    path, out_json, key, steps = argv[0], argv[1], argv[2], float(argv[3])
    dom = argv[4] if len(argv) > 4 else None
    dom_flop = float(argv[5]) if len(argv) > 5 else None
    keep, counts = graph_step_dispatches(path, int(steps)) if graph else (None, None)
    per = defaultdict(lambda: defaultdict(float))       # (dispatch id) -> counter -> value
    names = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            d = int(r.get("Dispatch_Id") or r.get("Correlation_Id"))
            if keep is not None and d not in keep:
                continue
            per[d][r["Counter_Name"]] += float(r["Counter_Value"])
            names[d] = kernel_key(r["Kernel_Name"])
    busy = sum(v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) for v in per.values())
    gui = sum(v.get("GRBM_GUI_ACTIVE", 0.0) for v in per.values())
    rec = {"dispatches": len(per), "steps": steps,
           "scope": (f"the last {int(steps)} graph-replayed steps ({counts} launches each)" if graph
                     else "every dispatch of the profiled program"),
           "mfma_busy_cycles_per_step": busy / steps, "kernel_cycles_per_step": gui / 8 / steps,
           "step_mfma_busy_frac": busy / (1024.0 * gui / 8) if gui else None,
           "formula": "sum SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x sum GRBM_GUI_ACTIVE / 8) over the step's dispatches"}
    by_k = defaultdict(lambda: [0.0, 0.0, 0])
    for d, v in per.items():
        k = by_k[names[d]]
        k[0] += v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        k[1] += v.get("GRBM_GUI_ACTIVE", 0.0)
        k[2] += 1
    top = sorted(by_k.items(), key=lambda kv: -kv[1][1])[:12]
    rec["kernels"] = {n: {"dispatches": c, "mfma_busy_frac": b / (1024.0 * g / 8) if g else None,
                          "share_of_kernel_cycles": g / gui if gui else None} for n, (b, g, c) in top}
    if dom:
        ents = [(n, v) for n, v in by_k.items() if dom in n]
        if ents and dom_flop:
            b = sum(v[0] for _, v in ents)
            c = sum(v[2] for _, v in ents)
            rec["calibration"] = {"kernel": dom, "measured_busy_per_launch": b / c,
                                  "algorithmic_mfma_cycles_per_launch": dom_flop / 1024.0,
                                  "ratio": (b / c) / (dom_flop / 1024.0)}
    data = {}
    if os.path.exists(out_json):
        with open(out_json) as fh:
            data = json.load(fh)
    data[key] = rec
    with open(out_json, "w") as fh:
        json.dump(data, fh, indent=1, sort_keys=True)
    print(json.dumps({k: rec[k] for k in ("dispatches", "step_mfma_busy_frac")}), rec.get("calibration"))


if __name__ == "__main__":
    main()
