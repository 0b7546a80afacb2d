#!/usr/bin/env python3
"""Runs the hipSPARSE comparison (tools/hipsparse_cmp.cpp; SURVEY.md §8f rank
3, hipsparse-spmv/spmv.cu:151-180 is the reference's driver) on the BASELINE
configurations: writes each config matrix (with its CSR-3 maps, so libhspmv
runs the kernel the bench runs) as an hspmv binary cache and calls the
comparison binary on it: warm and cold (Infinity Cache evicted) event-timed
launches of libhspmv and of hipsparseSpMV ALG_DEFAULT / CSR_ALG1 / CSR_ALG2
on the same device x, one JSON line each.

    python heterogeneous-spmv_amd/tools/hipsparse_cmp.py [--configs c2,c3,c4,c5]
           [--iters 30] [--cold 10] [--dump DIR] [--out F.jsonl]
"""
import argparse
import json
import subprocess
import sys
import tempfile
from pathlib import Path

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent))
sys.path.insert(0, str(HERE))

from sweep import build  # noqa: E402  (imports torch before libhspmv)

import hspmv  # noqa: E402

BIN = HERE.parent / "build" / "hipsparse_cmp"


def compare(cfg, A, maps, desc, iters=30, cold=10, dump_dir=None, tmp=None, timeout=300):
    """One matrix: returns the JSON records (hspmv first, then each hipSPARSE
    algorithm); with dump_dir the y vectors land in dump_dir/<cfg>_<impl>.bin."""
    with tempfile.TemporaryDirectory(dir=tmp or "/tmp") as td:
        path = Path(td) / f"{cfg}.bin"
        hspmv.save_bin(path, A, maps)
        args = [str(BIN), str(path), str(iters), str(cold)]
        if dump_dir is not None:
            args.append(str(Path(dump_dir) / cfg))
        p = subprocess.run(args, capture_output=True, text=True, timeout=timeout)
        if p.returncode != 0:
            raise RuntimeError(f"hipsparse_cmp {cfg}: rc {p.returncode}\n{p.stdout}\n{p.stderr[-4000:]}")
    out = []
    for line in p.stdout.splitlines():
        if line.startswith("{"):
            d = json.loads(line)
            d["config"] = cfg
            d["desc"] = desc
            out.append(d)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c2,c3,c4,c5")
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--cold", type=int, default=10)
    ap.add_argument("--dump", default="")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    out = []
    for cfg in a.configs.split(","):
        A, maps, desc = build(cfg)
        for d in compare(cfg, A, maps, desc, a.iters, a.cold, a.dump or None):
            out.append(d)
            print(json.dumps(d), flush=True)
    if a.out:
        Path(a.out).write_text("".join(json.dumps(d) + "\n" for d in out))


if __name__ == "__main__":
    main()
