"""The committed round evidence is self-consistent (CPU only, no GPU call): the closing bench line keeps the
bench.py contract (BASELINE.json's metric, roofline and cpu_baseline objects, frac = achieved / peak), its
`traffic` is the PMC figure of `pmc_traffic.json` for the same kernel family, and that JSON is reproduced from
the raw counter CSVs committed beside it by the same tools (tools/pmc_traffic.py, tools/pmc_mfma.py)."""
import glob
import gzip
import json
import os
import shutil
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))


def _latest_round():
    rounds = sorted(d for d in glob.glob(os.path.join(REPO, "profiles", "r[0-9][0-9]"))
                    if os.path.exists(os.path.join(d, "bench_default.json")))
    if not rounds:
        pytest.skip("no profiles/rNN/bench_default.json")
    return rounds[-1]


@pytest.fixture(scope="module")
def line():
    with open(os.path.join(_latest_round(), "bench_default.json")) as f:
        return json.loads(f.read().strip().splitlines()[-1])


def test_bench_line_contract(line):
    with open(os.path.join(REPO, "BASELINE.json")) as f:
        base = json.load(f)
    assert line["metric"] == base["metric"]
    for k in ("value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in line, k
    assert line["n_gpus"] == 1 and line["higher_is_better"] is True and line["scaling"] in ("weak", "strong")
    assert "workload" in line["config"] and line["data"].startswith("synthetic")
    # value = frames per step / step time
    assert line["value"] == pytest.approx(line["config"]["global_units_per_step"] / (line["ms_per_step"] * 1e-3),
                                          rel=2e-3)
    r = line["roofline"]
    assert r["bound"] in ("hbm", "mfma") and r["unit"] == ("GB/s" if r["bound"] == "hbm" else "TFLOP/s")
    assert r["frac"] == pytest.approx(r["achieved"] / r["peak"], rel=1e-3)
    per_launch = r["algorithmic_bytes_per_launch"] if r["bound"] == "hbm" else r["algorithmic_flop_per_launch"]
    scale = 1e9 if r["bound"] == "hbm" else 1e12
    assert r["achieved"] == pytest.approx(per_launch / (r["avg_launch_us"] * 1e-6) / scale, rel=2e-3)
    c = line["cpu_baseline"]
    assert c["kind"] in ("port", "reference") and c["cores"] >= 1 and c["value"] > 0 and c["sample"]


def test_traffic_matches_pmc_json(line):
    r = line["roofline"]
    if r["traffic"] is None:
        pytest.skip("no PMC traffic on this line")
    with open(os.path.join(_latest_round(), "pmc_traffic.json")) as f:
        pmc = json.load(f)
    kern = pmc["extract"]["kernels"][r["kernel"]]
    # the bench reads the JSON committed when it ran; the closing bundle regenerates it afterwards from the same
    # kernels, so the two collections agree to counter noise
    assert r["traffic"] == pytest.approx(kern["hbm_bytes_per_launch"], rel=0.01)
    assert kern["hbm_bytes_per_launch"] >= 0.9 * r["algorithmic_bytes_per_launch"]


def test_pmc_traffic_reproduced_from_committed_csvs(tmp_path):
    import pmc_traffic

    with open(os.path.join(_latest_round(), "pmc_traffic.json")) as f:
        entry = json.load(f)["extract"]
    csvs = []
    for src in entry["source"]:
        path = os.path.join(REPO, src)
        assert os.path.exists(path), src
        out = tmp_path / os.path.basename(src).replace(".gz", "")
        with gzip.open(path, "rb") as fi, open(out, "wb") as fo:
            shutil.copyfileobj(fi, fo)
        csvs.append(str(out))
    steps = int(entry["scope"].split()[2]) if entry["scope"].startswith("the last") else 0
    keep_f = pmc_traffic.graph_step_dispatches(csvs[0], steps)[0] if steps else None
    keep_w = pmc_traffic.graph_step_dispatches(csvs[1], steps)[0] if steps else None
    fetch = pmc_traffic.per_kernel(csvs[0], "FETCH_SIZE", keep_f)
    write = pmc_traffic.per_kernel(csvs[1], "WRITE_SIZE", keep_w)
    for name, k in entry["kernels"].items():
        f, w = fetch[name], write[name]
        assert len(f) == k["dispatches"], name
        got = (2.0 * sum(f) / len(f) + sum(w) / len(w)) * 1024.0
        assert got == pytest.approx(k["hbm_bytes_per_launch"], abs=1.0), name


def test_pmc_mfma_reproduced_from_committed_csv(tmp_path):
    import subprocess

    rdir = _latest_round()
    with open(os.path.join(rdir, "pmc_mfma.json")) as f:
        want = json.load(f)["extract_fp16"]
    src = os.path.join(rdir, "pmc", "extract_fp16_graph_m.csv.gz")
    csv_path = tmp_path / "m.csv"
    with gzip.open(src, "rb") as fi, open(csv_path, "wb") as fo:
        shutil.copyfileobj(fi, fo)
    out = tmp_path / "mfma.json"
    args = [sys.executable, os.path.join(REPO, "tools", "pmc_mfma.py"), str(csv_path), str(out), "extract_fp16",
            str(int(want["steps"]))] + (["--graph"] if want["scope"].startswith("the last") else [])
    r = subprocess.run(args, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    with open(out) as f:
        got = json.load(f)["extract_fp16"]
    assert got["dispatches"] == want["dispatches"]
    assert got["step_mfma_busy_frac"] == pytest.approx(want["step_mfma_busy_frac"], rel=1e-9)


def test_kernel_family_folds_gemm_pk_perm():
    """gemm_pk's PERM template argument (the W-row permutation for 16-byte epilogue operands) is one family with
    the unpermuted instantiation, as bench.py's svk_last_kernel name reports it; other kernels keep their names."""
    import pmc_traffic

    base = "gemm_pk<_Float16, PkCfg<128, 128, 2, 2, 2>, false, true, 0, false, false"
    assert pmc_traffic._family(base + ", true>") == base + ">"
    assert pmc_traffic._family(base + ", false>") == base + ">"
    assert pmc_traffic._family(base + ">") == base + ">"
    assert pmc_traffic._family("attn_block<_Float16, 1, 8, 256>") == "attn_block<_Float16, 1, 8, 256>"
