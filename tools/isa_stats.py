#!/usr/bin/env python3
"""tools/isa_stats.py — static instruction mix of each kernel in a hipcc -save-temps gfx950 .s."""
import re
import sys


def main(path, filt=""):
    lines = open(path).read().split("\n")
    starts = [i for i, l in enumerate(lines) if re.match(r"^(_Z\S+):\s*(;.*)?$", l)]
    starts.append(len(lines))
    for a, b in zip(starts, starts[1:]):
        name = lines[a].split(":")[0]
        if filt not in name:
            continue
        ins = []
        for l in lines[a + 1:b]:
            t = l.strip()
            if not t or t.startswith((".", ";")) or t.endswith(":"):
                continue
            op = t.split()[0]
            if re.match(r"^[a-z_0-9]+$", op):
                ins.append(op)
            if op == "s_endpgm":
                break
        c = lambda p: sum(1 for i in ins if i.startswith(p))
        print(f"{name[:70]:70s} total {len(ins):5d} valu {c('v_'):5d} salu {c('s_'):4d} "
              f"vmem {c('global_') + c('buffer_'):4d} lds {c('ds_'):3d} f64 {sum('f64' in i for i in ins):3d} "
              f"br {c('s_cbranch'):3d} saveexec {sum('saveexec' in i for i in ins):3d}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
