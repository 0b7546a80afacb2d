"""The sweep harness (tools/run_sweep.py) writes the reference's run_scripts CSV
layout (run_scripts/run_norm.py:94-115: kernel, mat, sch, threads, min, max,
avg,) from the drivers' stdout.  The CPU test drives it with stand-in drivers
that print a fixed report; the GPU test runs the real drivers."""
import os
import stat
import sys

import pytest

from conftest import GOLDEN, REPO

sys.path.insert(0, str(REPO / "heterogeneous-spmv_amd" / "tools"))
import run_sweep  # noqa: E402

REPORT = """Kernel: stream
TimeMin: 1.5e-05
TimeMax: 2.25e-05
TimeAvg: 1.75e-05
Number Wrong: 0
GFLOPs: 512.5
GBps: 4100
Check: PASS maxrel=0
"""


def fake_build(tmp_path, report=REPORT, rc=0):
    b = tmp_path / "build"
    b.mkdir()
    for drv in ("spmv-csr", "spmv-csrk"):
        p = b / drv
        # echoes its argv on stderr so the test can check the command line
        p.write_text(f"#!/bin/sh\necho \"$@\" 1>&2\ncat <<'EOF'\n{report}EOF\nexit {rc}\n")
        p.chmod(p.stat().st_mode | stat.S_IXUSR)
    return b


def mats(tmp_path):
    d = tmp_path / "mats"
    d.mkdir()
    for name in ("a.csr", "b.csr3", "ignored.txt"):
        (d / name).write_text("")
    return d


def test_parse_times_matches_run_norm_slicing():
    assert run_sweep.parse_times(REPORT) == ["1.5e-05", "2.25e-05", "1.75e-05"]
    assert run_sweep.parse_times("TimeMin: 1\nTimeMax: 2\n") is None
    assert run_sweep.parse_key(REPORT, "GBps:") == "4100"


def test_csv_rows_and_run_logs(tmp_path):
    b, d, out = fake_build(tmp_path), mats(tmp_path), tmp_path / "out"
    rc = run_sweep.main(["--matrices", str(d), "--build", str(b), "--out", str(out),
                         "--schedules", "auto,stream", "--gpus", "1,2", "--num-runs", "5"])
    assert rc == 0
    rows = (out / "sweep.csv").read_text().splitlines()
    assert len(rows) == 2 * 2 * 2 * 2  # drivers x matrices x schedules x gpus
    assert rows[0] == ("spmv-csr, a.csr, auto, 1, 1.5e-05, 2.25e-05, 1.75e-05, 512.5, 4100, "
                       "PASS, ")
    log = (out / "runs" / "spmv-csrk" / "b.csr3_stream_2.txt").read_text()
    assert "5 --kernel stream --gpus 2 --dtype f64" in log and "TimeAvg:" in log


def test_tuning_sizes_column_only_for_csrk(tmp_path):
    b, d, out = fake_build(tmp_path), mats(tmp_path), tmp_path / "out"
    run_sweep.main(["--matrices", str(d), "--build", str(b), "--out", str(out),
                    "--sizes", "20x10,7x8"])
    rows = (out / "sweep.csv").read_text().splitlines()
    csrk = [r for r in rows if r.startswith("spmv-csrk")]
    assert len(csrk) == 4 and all(r.split(", ")[4] in ("(20 10)", "(7 8)") for r in csrk)
    assert len([r for r in rows if r.startswith("spmv-csr,")]) == 2
    log = (out / "runs" / "spmv-csrk" / "a.csr_auto_1_7x8.txt").read_text()
    assert f"{d / 'a.csr'} 20 7 8 --gpus 1" in log


def test_failed_runs_are_skipped(tmp_path):
    b, d, out = fake_build(tmp_path, report="read failed\n", rc=1), mats(tmp_path), tmp_path / "o"
    assert run_sweep.main(["--matrices", str(d), "--build", str(b), "--out", str(out)]) == 1
    assert not (out / "sweep.csv").exists()


@pytest.mark.gpu
def test_sweep_on_golden_matrices(tmp_path):
    d = tmp_path / "mats"
    d.mkdir()
    for name in ("lap32.mtx.rcm.csr", "powerlaw1500.csr3"):
        os.symlink(GOLDEN / name, d / name)
    out = tmp_path / "out"
    rc = run_sweep.main(["--matrices", str(d), "--out", str(out), "--num-runs", "5",
                         "--schedules", "auto,stream", "--sizes", "8x4"])
    assert rc == 0
    rows = [r.split(", ") for r in (out / "sweep.csv").read_text().splitlines()]
    assert len(rows) == 8
    for r in rows:
        t = [float(v) for v in (r[5:8] if r[0] == "spmv-csrk" else r[4:7])]
        assert 0 < t[0] <= t[2] <= t[1]
        assert r[-2] == "PASS"
    # the summation contracts as schedules; the serial one also bitwise
    out2 = tmp_path / "out2"
    rc = run_sweep.main(["--matrices", str(d), "--out", str(out2), "--num-runs", "3", "--drivers", "spmv-csr",
                         "--schedules", "ordered,reproducible,serial"])
    assert rc == 0
    rows = [r.split(", ") for r in (out2 / "sweep.csv").read_text().splitlines()]
    assert len(rows) == 2 * 3 and all(r[-2] == "PASS" for r in rows), rows
    logs = list((out2 / "runs" / "spmv-csr").glob("*_serial_*.txt"))
    assert logs and all("Bitwise: 0 rows differ" in f.read_text() for f in logs)


def test_mtx_inputs_are_converted_first(tmp_path):
    """--mtx: the reference's conversion steps (converter.m, convert-all.sh)
    with the real host-only converters, then the (stand-in) drivers."""
    import scipy.io
    import scipy.sparse as sp
    src = tmp_path / "mm"
    src.mkdir()
    S = sp.random(300, 300, density=0.02, random_state=1, format="csr") + sp.eye(300)
    scipy.io.mmwrite(str(src / "r300.mtx"), S)
    b = fake_build(tmp_path)
    for tool in ("mtx2csr", "reformat-auto"):
        (b / tool).symlink_to(REPO / "heterogeneous-spmv_amd" / "build" / tool)
    out = tmp_path / "out"
    rc = run_sweep.main(["--mtx", str(src), "--csr3", "--build", str(b), "--out", str(out),
                         "--drivers", "spmv-csr", "--num-runs", "3"])
    assert rc == 0
    names = sorted(p.name for p in (out / "matrices").iterdir())
    assert names == ["r300.mtx.csr", "r300.mtx.rcm.csr", "r300.mtx.rcm.csr3"]
    rows = (out / "sweep.csv").read_text().splitlines()
    assert [r.split(", ")[1] for r in rows] == names
