#!/usr/bin/env python3
"""Runs the hipSPARSE comparison (tools/hipsparse_cmp.cpp) on the BASELINE
configurations: writes each config matrix as an hspmv binary cache and calls
the comparison binary on it.

    python heterogeneous-spmv_amd/tools/hipsparse_cmp.py [--configs c2,c3,c4,c5] [--out F.jsonl]
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

import hspmv  # noqa: E402
from sweep import build  # noqa: E402

BIN = HERE.parent / "build" / "hipsparse_cmp"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c2,c3,c4,c5")
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    out = []
    with tempfile.TemporaryDirectory(dir="/tmp") as td:
        for cfg in a.configs.split(","):
            A, maps, desc = build(cfg)
            path = Path(td) / f"{cfg}.bin"
            hspmv.save_bin(path, A)
            p = subprocess.run([str(BIN), str(path), str(a.iters)], capture_output=True, text=True,
                               timeout=600)
            if p.stderr:
                print(p.stderr[-20000:], file=sys.stderr)
            if p.returncode != 0:
                print(p.stdout, file=sys.stderr)
                raise SystemExit(p.returncode)
            for line in p.stdout.splitlines():
                d = json.loads(line)
                d["config"] = cfg
                d["desc"] = desc
                out.append(d)
                print(json.dumps(d), flush=True)
            path.unlink()
    if a.out:
        Path(a.out).write_text("".join(json.dumps(d) + "\n" for d in out))


if __name__ == "__main__":
    main()
