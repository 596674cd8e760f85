"""HBM bytes per launch of the bench's kernel classes from two rocprofv3 --pmc passes.

python scripts/pmc_traffic.py <fetch counter_collection.csv> <write counter_collection.csv>

Corrections per /opt/skills/guides/MI355X_MICROARCH.md (HBM section): FETCH_SIZE (kilobytes,
from TCC_EA0_RDREQ x 64 B) reports half the bytes of wide coalesced reads on gfx950, so it is
doubled; WRITE_SIZE (kilobytes) is taken as is.  Infinity-Cache hits are counted, not excluded,
so these are memory-side (MALL + HBM) bytes.  Prints JSON keyed like bench.py's roofline classes.
"""
import csv
import json
import sys

CLASSES = {"gemm": ("gemm_kernel", "splitk_reduce_kernel"),
           "spmm": ("spmm_seg_kernel", "spmm_fix_kernel", "spmm_lane_kernel", "spmm_blk_kernel")}
PRIMARY = {"gemm": ("gemm_kernel",), "spmm": ("spmm_seg_kernel", "spmm_lane_kernel", "spmm_blk_kernel")}


def load(path, counter):
    out = []
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        out.append((name.split("<")[0], float(r["Counter_Value"])))
    return out


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    res = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE over `bench.py --steps 1 --warmup 1` (2 epochs + eval)",
           "correction": "bytes = 2 * FETCH_SIZE_KB * 1024 + WRITE_SIZE_KB * 1024 (gfx950 FETCH_SIZE halving)"}
    for cls, names in CLASSES.items():
        f = sum(v for n, v in fetch if n in names) * 1024 * 2
        w = sum(v for n, v in write if n in names) * 1024
        launches = sum(1 for n, _ in fetch if n in PRIMARY[cls])
        res[cls] = {"launches": launches, "fetch_bytes": f, "write_bytes": w,
                    "traffic_per_launch": (f + w) / max(launches, 1)}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
