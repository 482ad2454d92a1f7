#!/usr/bin/env python3
"""Summarises interleaved A/B rounds of tools/kbench.py lines (JSON per line, keyed by `tag`):
per tag, the wall time per frame (no events) and the event span of every round.

  python tools/ab_summary.py gpurun_out/r06c/share_ab.jsonl
"""
from __future__ import annotations

import collections
import json
import sys


def main():
    d = collections.defaultdict(list)
    for path in sys.argv[1:]:
        for line in open(path):
            if line.startswith("{"):
                r = json.loads(line)
                d[r["tag"]].append((r.get("wall_us_no_events"), r.get("med_us")))
    for k in sorted(d):
        print(f"{k:50s} wall us/frame {[x[0] for x in d[k]]}  span us {[x[1] for x in d[k]]}")


if __name__ == "__main__":
    main()
