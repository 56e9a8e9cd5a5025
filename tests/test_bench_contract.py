"""The BENCH line's contract (the driver parses bench.py's one JSON line), checked on the line the
final round-6 build printed on the MI355X box (profiles/r06/bench.json) and on the code that makes
it: every required key, the roofline and cpu_baseline objects, and their internal consistency."""
import json
import os

from conftest import ROOT

REQUIRED = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
            "scaling", "vs_baseline", "dtype", "data", "config"}


def _line():
    with open(os.path.join(ROOT, "profiles", "r06", "bench.json")) as f:
        lines = [ln for ln in f.read().splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    return json.loads(lines[0])


def test_bench_line_has_the_contract_keys():
    d = _line()
    assert REQUIRED <= set(d)
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        base = json.load(f)
    assert d["metric"] == base["metric"] and d["unit"] == "GiB/s"
    assert d["higher_is_better"] is True and d["scaling"] == "weak" and d["vs_baseline"] is None
    assert d["n_gpus"] == 1 and "workload" in d["config"] and "model" not in d["config"]
    # value = N x 0.25 GiB per step / step time
    assert abs(d["value"] - 0.25 * d["n_gpus"] / (d["ms_per_step"] * 1e-3)) / d["value"] < 0.01


def test_roofline_object():
    r = _line()["roofline"]
    assert {"bound", "achieved", "peak", "unit", "frac", "traffic"} <= set(r)
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    # algorithmic bytes per launch (20 B/elem x 64 Mi) / kernel time = achieved
    assert r["algorithmic_bytes_per_launch"] == 20 * 65536 * 1024
    # PMC traffic within 0.1 % of the algorithmic bytes: no wasted re-reads
    assert abs(r["traffic"] / r["algorithmic_bytes_per_launch"] - 1) < 1e-3


def test_cpu_baseline_object():
    c = _line()["cpu_baseline"]
    assert {"value", "unit", "cores", "kind", "sample"} <= set(c)
    assert c["kind"] in ("port", "reference") and c["cores"] >= 1 and c["unit"] == "GiB/s"


def test_rank_devices_reported():
    """Every rank's observed device: devices_used is the distinct count of what
    the ranks reported."""
    d = _line()
    rd = d["rank_devices"]
    assert len(rd) == d["n_gpus"] and all(r["pci"] for r in rd)
    assert d["devices_used"] == len({(r["host"], r["pci"]) for r in rd})


def test_rank_devices_carry_each_ranks_kernels():
    """Each rank's own kernel times and roofline fractions, beside its device:
    frac = kernel bytes / time / peak, so a slow rank is visible in the line, not only the max."""
    d = _line()
    for r in d["rank_devices"]:
        km, fr = r["kernels_ms"], r["roofline_frac"]
        assert km["encode"] > 0 and km["decode"] > 0 and r["step_ms"] > 0
        for k in ("encode", "decode"):
            want = 20 * 65536 * 1024 / (km[k] * 1e-3) / 1e9 / 8000.0
            assert abs(fr[k] - want) < 2e-3 * want + 1e-3, (k, fr[k], want)


def test_config3_both_layouts_reported():
    c3 = _line()["config3"]
    assert c3["roundtrip_ok"] and c3["views"]["roundtrip_ok"]
    assert c3["table_entries"] == {"encode": 4096, "decode": 4096}
    assert c3["views"]["table_entries"] == {"encode": 1, "decode": 1}
    # per-launch batched kernel times and the tile each direction ran with
    assert c3["kernels_ms"]["encode"] > 0 and c3["kernels_ms"]["decode"] > 0
    assert set(c3["tile_lanes_pairs"]) == {"encode", "decode"}


def test_pmc_traffic_names_the_shipping_library():
    """profiles/pmc_traffic.json (bench.py's roofline.traffic source) was measured with the library
    this tree builds (efl_version's source hash), so the bench line's traffic_source and library
    agree."""
    import subprocess
    with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as f:
        tr = json.load(f)
    h = subprocess.check_output(["make", "-s", "-C", os.path.join(ROOT, "elastic-federated-learning-solution_amd"),
                                 "src-hash"], text=True).strip()
    assert tr["library"].endswith("src " + h), (tr["library"], h)
    assert tr["elements"] == 65536 * 1024


def _src_hash():
    import subprocess
    return subprocess.check_output(["make", "-s", "-C", os.path.join(ROOT, "elastic-federated-learning-solution_amd"),
                                    "src-hash"], text=True).strip()


def test_records_come_from_the_shipping_library():
    """The round's BENCH line and Stage P report were measured with the library this tree builds,
    and the Stage P report carries the GMP CPU baseline of the same run (bench hygiene)."""
    h = _src_hash()
    assert _line()["library"].endswith("src " + h)
    with open(os.path.join(ROOT, "profiles", "r06", "bench_stage_p.jsonl")) as f:
        lines = [json.loads(ln) for ln in f if ln.startswith("{")]
    assert len(lines) == 3
    for d in lines:
        assert d["library"].endswith("src " + h), d["library"]
        cb = d["cpu_baseline"]
        assert cb and cb["kind"] in ("port", "reference") and cb["encrypt"] > 0 and cb["decrypt"] > 0
        assert d["encrypt"]["vs_cpu"] > 1 and d["decrypt"]["vs_cpu"] > 1
