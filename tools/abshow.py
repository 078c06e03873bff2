#!/usr/bin/env python3
"""tools/abshow.py — one line per variant of tools/ab_schedule.py result files."""
import json
import sys

for f in sys.argv[1:]:
    txt = "".join(l for l in open(f) if "amdgpu.ids" not in l)
    try:
        d = json.loads(txt)
    except ValueError:
        print(f, "unparsable:", txt[-300:])
        continue
    for k, v in d["results"].items():
        print(f"{f.split('/')[-1]:22s} {k:24s} median {v['median_ms']:9.2f} ms  {v['mrays_per_s']:9.1f} Mrays/s  "
              f"segs {v['segments']}  same {v['equal_pixel_frac']:.4f}  {v['kernel_ms']}")
