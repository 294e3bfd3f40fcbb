#!/usr/bin/env python3
"""Dev: the HBM ceiling table for the headline's traffic (15.73 GB read +
1.81 GB written, 8.7 : 1) from tools/ubench/hbm_ceiling.hip runs on several
boxes (the committed logs below), one row per form and a column per box, and
the practical ceiling bench.py quotes as roofline.practical: the median over
boxes of the best contiguous-tile form.

    python3 tools/dev/ceiling_table.py > profiles/r6_hbm_ceiling.json
"""
import json
import os
import re
import statistics

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
LOGS = {   # box label -> committed ubench log (profiles/), its memory vendor where recorded
    "A": ("r6_a_hbm_ceiling.txt", None),
    "B": ("r6_b_hbm_bands.txt", None),
    "C": ("r6_c_hbm_adj.txt", None),
    "D": ("r6_f_hbm_store_forms_samsung.txt", "samsung"),
    "E": ("r6_g_hbm_ceiling.txt", "samsung"),
    "F": ("r6_z_hbm_ceiling.txt", "samsung"),   # the round-end passes' boxes (profiles/r6_z_* ... r6_z5_*)
    "G": ("r6_z2_hbm_ceiling.txt", "samsung"),
    "H": ("r6_z3_hbm_ceiling.txt", "samsung"),
    "I": ("r6_z4_hbm_ceiling.txt", "samsung"),
    "J": ("r6_z5_hbm_ceiling.txt", "samsung"),
}
LINE = re.compile(r"^(.*?)\s+best\s+([\d.]+) ms\s+mean\s+([\d.]+) ms\s+([\d.]+) GB/s")


def main():
    rows, vendors = {}, {}
    for box, (f, vendor) in LOGS.items():
        vendors[box] = vendor
        for ln in open(os.path.join(ROOT, "profiles", f)):
            m = LINE.match(ln.strip())
            if m:
                rows.setdefault(m.group(1).strip(), {})[box] = {"best_ms": float(m.group(2)),
                                                                "GBps": float(m.group(4))}
    tile = [v["GBps"] for b, v in rows.get("tile 8.7:1 ld nt   st nt", {}).items()]
    same = ("prod DMA + b64 stores", "prod LDS-DMA nt + b64 stores", "band1 DMA nt + b64 stores")   # one form, three names
    prod = {}
    for name in same:
        for b, v in rows.get(name, {}).items():
            prod.setdefault(b, v["best_ms"])
    out = {
        "source": f"tools/ubench/hbm_ceiling.hip on {len(LOGS)} boxes (profiles/r6_*_hbm_*.txt); tools/dev/ceiling_table.py",
        "bytes": {"read": 15728640000, "write": 1806336000},
        "boxes": vendors,
        "rows": rows,
        "practical": {
            "form": "mix-shaped contiguous tiles, nt loads and nt stores (k_tile<1,1>): 8 tracks x 10 KiB read and "
                    "9.4 KiB written per workgroup, the best form measured for this byte mix",
            "GBps_median": statistics.median(tile) if tile else None,
            "GBps_per_box": {b: v["GBps"] for b, v in rows.get("tile 8.7:1 ld nt   st nt", {}).items()},
        },
        "product_geometry_ms": {"rows": "the fused kernel's own read stream (2048 waves x 64 streams of 256-B "
                                        "pieces) with its b64 output stores, no compute",
                                "best_ms_per_box": prod},
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
