#!/usr/bin/env python3
"""Pretty-print sweep JSON lines: show_sweep.py FILE.jsonl [FILE2.jsonl ...]"""
import json
import sys

for path in sys.argv[1:]:
    for line in open(path):
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        print(f"{d['config']:3} {d['variant']:22} ok={d['ok']!s:5} t_min={d['t_min_us']:9.2f}us "
              f"t_avg={d['t_avg_us']:9.2f}us GB/s={d['gbps_min']:7.1f} frac={d['frac_peak']:.3f} "
              f"u={d.get('chunk_u')} W={d.get('waves_per_block')} split={d.get('n_split_rows')}")
