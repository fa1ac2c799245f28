"""CPU: the measurement tooling behind bench.py's VALU roofline — tools/pmc_valu.py over a synthetic rocprofv3 counter
CSV, bench.valu_roofline's measured-issue band, and bench.pmc_pass picking the newest committed pass."""
import csv
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def _counter_csv(path, rows):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Dispatch_Id", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for d, (kernel, counters) in enumerate(rows):
            for name, v in counters.items():
                w.writerow({"Kernel_Name": kernel, "Dispatch_Id": str(d), "Counter_Name": name, "Counter_Value": str(v)})


def test_pmc_valu_per_witness(tmp_path):
    # two batches (two k_load_values dispatches) of 4 witnesses: per-witness figures divide by 2 x 4
    rows = [("void pzk::k_load_values(pzk::Load const*)", {"SQ_INSTS_VALU": 8, "SQ_ACTIVE_INST_VALU": 8}),
            ("void pzk::k_emit_sha<16, 0>(pzk::DevLayout)", {"SQ_INSTS_VALU": 800, "SQ_ACTIVE_INST_VALU": 800,
                                                            "SQ_INSTS_VALU_INT64": 80, "SQ_INSTS_VALU_INT32": 400}),
            ("void pzk::k_load_values(pzk::Load const*)", {"SQ_INSTS_VALU": 8, "SQ_ACTIVE_INST_VALU": 8}),
            ("void pzk::k_emit_sha<16, 0>(pzk::DevLayout)", {"SQ_INSTS_VALU": 800, "SQ_ACTIVE_INST_VALU": 800,
                                                            "SQ_INSTS_VALU_INT64": 80, "SQ_INSTS_VALU_INT32": 400}),
            ("at::native::elementwise_kernel(...)", {"SQ_INSTS_VALU": 1000})]  # not ours: ignored
    src, out = tmp_path / "c.csv", tmp_path / "v.json"
    _counter_csv(src, rows)
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "pmc_valu.py"), str(src), "4", "1000", str(out)],
                       capture_output=True, text=True, check=True)
    assert "k_emit_sha" in r.stdout
    v = json.load(open(out))
    sha = v["kernels"]["k_emit_sha"]
    assert sha["valu_insts_per_witness"] == 200.0 and sha["valu_cycles_per_witness"] == 800.0
    assert sha["int64_per_witness"] == 20.0 and sha["int32_per_witness"] == 100.0
    assert v["valu_insts_per_witness"] == 202.0
    assert "k_load_values" in v["kernels"] and not any(k.startswith("at::") for k in v["kernels"])
    assert v["valu_cycle_frac"] == pytest.approx(808 * 1000 / (256 * 4 * 2.4e9), abs=1e-3)


def test_valu_roofline_measured_issue_band(tmp_path):
    d = tmp_path / "pmc_x"
    d.mkdir()
    tj = {"workload": "w", "layout_key": "O0", "valu_insts_per_witness": 1000.0,
          "kernels": {"k_a": {"valu_insts_per_witness": 1000.0}}}
    (d / "traffic.json").write_text(json.dumps(tj))
    (d / "valu.json").write_text(json.dumps({"valu_insts_per_witness": 1000.0,
                                             "kernels": {"k_a": {"int64_per_witness": 400.0}}}))
    r = bench.valu_roofline(tj, str(d / "traffic.json"), 1e6, 1)
    mi = r["measured_issue"]
    assert mi["int64_per_witness"] == 400.0 and mi["other_per_witness"] == 600.0
    lo = 1e6 * (400 / (bench.VALU_RATE_INT64_GIPS * 1e9) + 600 / (bench.VALU_RATE_SIMPLE_GIPS * 1e9))
    hi = 1e6 * (400 / (bench.VALU_RATE_INT64_GIPS * 1e9) + 600 / (bench.VALU_RATE_CARRY_GIPS * 1e9))
    assert mi["frac_lo"] == pytest.approx(lo, abs=1e-4) and mi["frac_hi"] == pytest.approx(hi, abs=1e-4)
    assert mi["frac_lo"] < mi["frac_hi"]
    # the nominal figure keeps its definition: instructions against one per 2 cycles per SIMD
    assert r["frac"] == pytest.approx(1000 * 1e6 / 1e9 / bench.VALU_PEAK_GIPS, abs=1e-4)
    # without a valu.json beside the pass the band is absent
    os.remove(d / "valu.json")
    assert "measured_issue" not in bench.valu_roofline(tj, str(d / "traffic.json"), 1e6, 1)


def test_pmc_pass_takes_the_newest_committed_pass():
    tf, tj = bench.pmc_pass(bench.CONFIG4_WORKLOAD, "O0")
    assert tj["workload"] == bench.CONFIG4_WORKLOAD and os.path.basename(os.path.dirname(tf)) >= "pmc_r6zg"
    assert os.path.exists(os.path.join(os.path.dirname(tf), "valu.json"))
    assert bench.pmc_pass("no such workload", "O0") is None
