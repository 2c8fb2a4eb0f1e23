"""The measurement tooling behind the bench line's roofline keys (CPU, synthetic inputs):
scripts/grbm_clock.py (GRBM_GUI_ACTIVE / 8 / dispatch wall per kernel), scripts/traffic_json.py
(the gfx950 FETCH_SIZE correction), and bench.py's lookups of the committed records."""
import csv
import json
import os
import subprocess
import sys

from conftest import REPO


def _write_csv(path, rows):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
        w.writeheader()
        w.writerows(rows)


def test_grbm_clock_per_kernel(tmp_path):
    # two dispatches of kernel K: 2.2e6 GUI-active cycles summed over 8 XCDs in 1 ms -> 275 MHz...
    # scaled: 8 * 2000e6 cycles/s * 0.010 s = 160e6 counts over a 10-ms dispatch = 2000 MHz
    cc = [{"Dispatch_Id": str(i), "Kernel_Name": "K", "Counter_Name": "GRBM_GUI_ACTIVE",
           "Counter_Value": str(8 * mhz * 1e6 * 0.010)} for i, mhz in ((1, 2000.0), (2, 2200.0))]
    cc += [{"Dispatch_Id": "1", "Kernel_Name": "K", "Counter_Name": "GRBM_COUNT", "Counter_Value": "1"}]
    kt = [{"Dispatch_Id": str(i), "Start_Timestamp": "0", "End_Timestamp": str(10_000_000)} for i in (1, 2)]
    _write_csv(tmp_path / "run_counter_collection.csv", cc)
    _write_csv(tmp_path / "run_kernel_trace.csv", kt)
    r = subprocess.run([sys.executable, os.path.join(REPO, "scripts", "grbm_clock.py"), str(tmp_path)],
                       capture_output=True, text=True, check=True)
    out = json.loads(r.stdout)["K"]
    assert out["dispatches"] == 2
    assert abs(out["grbm_clock_mhz_min_max"][0] - 2000.0) < 0.1 and abs(out["grbm_clock_mhz_min_max"][1] - 2200.0) < 0.1
    assert abs(out["ms_median"] - 10.0) < 1e-9


def test_traffic_record_correction(tmp_path):
    name = "void mcgmil::gate_fused_kernel<...>(mcgmil::GateParams)"
    json.dump({name: {"FETCH_SIZE": 1000.0}}, open(tmp_path / "fetch.json", "w"))
    json.dump({name: {"WRITE_SIZE": 500.0}}, open(tmp_path / "write.json", "w"))
    out = tmp_path / "t.json"
    subprocess.run([sys.executable, os.path.join(REPO, "scripts", "traffic_json.py"), str(tmp_path), str(out),
                    "cfg3", "cmd"], capture_output=True, text=True, check=True)
    rec = json.load(open(out))
    assert rec["hbm_bytes_per_launch"] == (2 * 1000 + 500) * 1024      # 2 x FETCH (KiB) + WRITE
    assert rec["path"] == "fused" and rec["config"]["bags"] == 512
    # H once + A once + Y for 512 bags of N = 2048, T = 100, C = 2, bf16
    assert rec["algorithmic_bytes_per_launch"] == 512 * 2048 * 512 * 2 + 100 * 2 * 512 * 2048 * 4 + 512 * 100 * 2 * 4


def test_bench_reads_the_committed_records():
    sys.path.insert(0, REPO)
    import bench
    t, src = bench.measured_traffic(2048, 100, 512, "bf16", 0, "fused")
    assert t and src.startswith("profiles/")
    mhz, src = bench.measured_grbm_clock("cfg3", "gate_fused_kernel")
    assert mhz and 1000.0 < mhz < 2600.0 and src.endswith("grbm_clock_cfg3.json")
    keys = bench.grbm_keys(1000.0, 2500.0, "cfg3", True)
    assert abs(keys["frac_at_grbm_clock"] - 1000.0 / (2500.0 * mhz / bench.MAX_CLOCK_MHZ)) < 1e-12
    # no calibration in this process: the measured-ceiling keys are present and null
    bench.CALIB.clear()
    assert bench.vs_measured(1000.0, "bf16") == {"measured_peak_tflops": None, "frac_of_measured": None}
