cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD --output-format csv -d gpurun_out/pmc_dw1 -o run -- python tools/dw_only.py > gpurun_out/pmc_dw1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmc_dw2 -o run -- python tools/dw_only.py > gpurun_out/pmc_dw2.log 2>&1 || exit 1
python - <<'PY'
import csv, collections
for d in ("pmc_dw1", "pmc_dw2"):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f"gpurun_out/{d}/run_counter_collection.csv")):
        if "dwconv" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        print(d, k, sum(v) / len(v))
PY
