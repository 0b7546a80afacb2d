#!/usr/bin/env python3
"""Sweep harness in the layout of the reference's run_scripts (SURVEY.md §8f
rank 4; run_scripts/run_norm.py:20-122, run_cuda_new.py, run_tuning.py): for
every driver x matrix x schedule x GPU count it runs

    <build>/<driver> <matrix> <num_runs> [sizes] [options]

keeps the driver's stdout in <out>/runs/<driver>/<mat>_<sch>_<gpus>.txt, reads
TimeMin/TimeMax/TimeAvg the way run_norm.py:94-107 does (find the key, take
the text from 8 characters after it to the end of the line) and appends one
CSV row per run to <out>/<record>:

    driver, mat, sch, gpus, min, max, avg, gflops, gbps, check,

-- the reference's columns (kernel, mat, sch, threads, min, max, avg) with the
GPU count in the threads column, plus the driver's GFLOPs / GBps lines and
its PASS/FAIL verdict against the serial CPU SpMV.  The
tuning mode (--sizes) adds the reference's "(ssrs srs)" column for spmv-csrk
manual sizes, as run_tuning.py:126 does.

    python heterogeneous-spmv_amd/tools/run_sweep.py --matrices DIR [--drivers spmv-csr,spmv-csrk]
        [--schedules auto,stream,csr3,vector,csort,ordered,reproducible,serial]
        [--gpus 1] [--num-runs 20]
        [--sizes 20x10,7x8] [--out DIR] [--record sweep.csv] [--timeout 600]
    python .../run_sweep.py --synthetic c2,c3 ...   # writes the configs as .csr first
    python .../run_sweep.py --mtx DIR [--csr3] ...   # SuiteSparse .mtx files first

--mtx runs the reference's conversion steps on every DIR/*.mtx before the
sweep, with this build's tools: mtx2csr (helpers/converter.m: X.mtx.csr and
the RCM-ordered X.mtx.rcm.csr) and, with --csr3, reformat-auto
(reformat-csr-to-csr3/convert-all.sh: X.mtx.rcm.csr3).

Matrices: every *.csr / *.csr3 / *.bin file in DIR (".csr3" carry their own
maps).  A run that times out is reported and skipped, like run_norm.py:86-89.
"""
from __future__ import annotations

import argparse
import subprocess
import sys
import time
from pathlib import Path

HERE = Path(__file__).resolve().parent
BUILD = HERE.parent / "build"

SCHEDULES = {  # schedule name -> driver options
    "auto": [], "stream": ["--kernel", "stream"], "csr3": ["--kernel", "csr3"],
    "vector": ["--kernel", "vector"], "nt": ["--kernel", "stream", "--nt"],
    "csort": ["--kernel", "csort"],
    # the summation contracts (hspmv_options.deterministic 1 / 2 / 3)
    "ordered": ["--deterministic"], "reproducible": ["--reproducible"], "serial": ["--serial"],
}


def parse_times(out: str):
    """run_norm.py:94-107: value = out[find(key) + 8 : end of that line]."""
    vals = []
    for key in ("TimeMin:", "TimeMax:", "TimeAvg:"):
        i = out.find(key)
        if i < 0:
            return None
        j = out.find("\n", i)
        vals.append(out[i + 8:j].strip())
    return vals


def parse_key(out: str, key: str) -> str:
    i = out.find(key)
    if i < 0:
        return ""
    j = out.find("\n", i)
    return out[i + len(key):j].strip()


def synthetic(configs, where: Path):
    sys.path.insert(0, str(HERE.parent))
    sys.path.insert(0, str(HERE))
    import hspmv
    from sweep import build
    where.mkdir(parents=True, exist_ok=True)
    for cfg in configs:
        A, maps, _ = build(cfg)
        if maps is not None:
            hspmv.write_csr3(where / f"{cfg}.csr3", A, maps)
        else:
            hspmv.write_csr(where / f"{cfg}.csr", A)


def convert_mtx(src: Path, where: Path, build: Path, csr3: bool, timeout: float) -> None:
    """converter.m + convert-all.sh for every src/*.mtx, into `where`."""
    where.mkdir(parents=True, exist_ok=True)
    for f in sorted(src.glob("*.mtx")):
        norm, rcm = where / f"{f.name}.csr", where / f"{f.name}.rcm.csr"
        subprocess.run([str(build / "mtx2csr"), str(f), str(norm), str(rcm)], check=True,
                       timeout=timeout)
        if csr3:
            subprocess.run([str(build / "reformat-auto"), str(rcm), str(where / f"{f.name}.rcm.csr3")],
                           check=True, capture_output=True, timeout=timeout)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--matrices", default="")
    ap.add_argument("--synthetic", default="", help="configs to generate (tools/sweep.py names)")
    ap.add_argument("--mtx", default="", help="directory of .mtx files to convert first")
    ap.add_argument("--csr3", action="store_true", help="with --mtx: also reformat-auto to .csr3")
    ap.add_argument("--drivers", default="spmv-csr,spmv-csrk")
    ap.add_argument("--schedules", default="auto")
    ap.add_argument("--gpus", default="1")
    ap.add_argument("--num-runs", type=int, default=20)
    ap.add_argument("--sizes", default="", help="spmv-csrk manual sizes, e.g. 20x10,7x8")
    ap.add_argument("--dtype", default="f64")
    ap.add_argument("--build", default=str(BUILD))
    ap.add_argument("--out", default="sweep_runs")
    ap.add_argument("--record", default="sweep.csv")
    ap.add_argument("--timeout", type=float, default=600.0)
    a = ap.parse_args(argv)
    out = Path(a.out)
    out.mkdir(parents=True, exist_ok=True)
    mdir = Path(a.matrices) if a.matrices else out / "matrices"
    if a.synthetic:
        synthetic(a.synthetic.split(","), mdir)
    if a.mtx:
        convert_mtx(Path(a.mtx), mdir, Path(a.build), a.csr3, a.timeout)
    mats = sorted(p for p in mdir.iterdir() if p.suffix in (".csr", ".csr3", ".bin"))
    record = out / a.record
    sizes = [tuple(s.split("x")) for s in a.sizes.split(",")] if a.sizes else [None]
    rows = 0
    for drv in a.drivers.split(","):
        print(f"-------{drv}------------", flush=True)
        rdir = out / "runs" / drv
        rdir.mkdir(parents=True, exist_ok=True)
        for mat in mats:
            for sch in a.schedules.split(","):
                for g in a.gpus.split(","):
                    for sz in (sizes if drv == "spmv-csrk" else [None]):
                        tag = f"{mat.name}_{sch}_{g}" + (f"_{sz[0]}x{sz[1]}" if sz else "")
                        cmd = [str(Path(a.build) / drv), str(mat), str(a.num_runs)]
                        if sz:
                            cmd += [sz[0], sz[1]]
                        cmd += SCHEDULES[sch] + ["--gpus", g, "--dtype", a.dtype]
                        print(f"{drv}_{tag}", flush=True)
                        tic = time.time()
                        try:
                            p = subprocess.run(cmd, capture_output=True, text=True,
                                               timeout=a.timeout)
                        except subprocess.TimeoutExpired:
                            print("Timeout:", mat, g, "Time:", time.time() - tic, flush=True)
                            continue
                        (rdir / f"{tag}.txt").write_text(p.stdout + p.stderr)
                        t = parse_times(p.stdout)
                        if p.returncode != 0 or t is None:
                            print(f"failed ({p.returncode}): {p.stderr.strip()[:200]}", flush=True)
                            continue
                        cols = [drv, mat.name, sch, g]
                        if sz:
                            cols.append(f"({sz[0]} {sz[1]})")
                        check = (parse_key(p.stdout, "Check:").split() or [""])[0]
                        cols += t + [parse_key(p.stdout, "GFLOPs:"), parse_key(p.stdout, "GBps:"),
                                     check]
                        line = ", ".join(cols) + ", \n"
                        with open(record, "a+") as f:
                            f.write(line)
                        print(line, end="", flush=True)
                        rows += 1
    return 0 if rows else 1


if __name__ == "__main__":
    sys.exit(main())
