"""Per-kernel-class memory-side bytes and MFMA utilisation from three rocprofv3 --pmc passes.

python scripts/pmc_summary.py <FETCH_SIZE csv> <WRITE_SIZE csv> <MFMA csv> "<bench command>"

Corrections per /opt/skills/guides/MI355X_MICROARCH.md (HBM section): FETCH_SIZE (kilobytes, from
TCC_EA0_RDREQ x 64 B) reports half the bytes of wide coalesced reads on gfx950, so it is doubled;
WRITE_SIZE (kilobytes) is taken as is.  Infinity-Cache hits are counted, not excluded, so these are
memory-side (MALL + HBM) bytes, an upper bound on HBM bytes.
MFMA utilisation of a class = sum SQ_VALU_MFMA_BUSY_CYCLES / (SIMDs per XCD-cycle x sum GRBM_GUI_ACTIVE):
GRBM_GUI_ACTIVE is summed over the 8 XCDs (= 8 x dispatch cycles) and the busy cycles over all
1,024 SIMDs, so the denominator is 128 x GRBM_GUI_ACTIVE.  The raw sums are kept beside it.
The JSON carries the SHA-256 of gmr/libgmr_hip.so so bench.py only uses it for the same build.
"""
import csv
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLASSES = {"gemm": ("gemm_kernel", "gemm_glds_kernel", "splitk_reduce_kernel"),
           "gemm_x6": ("gemm_x6_kernel", "split3_planes_kernel"),
           "spmm": ("spmm_seg_kernel", "spmm_fix_kernel", "spmm_lane_kernel", "spmm_lane_jobs_kernel",
                    "lane_fix_kernel", "lane_fix_jobs_kernel", "spmm_blk_kernel", "spmm_chunk_kernel", "spmm_side_kernel",
                    "spmm_side_jobs_kernel"),
           "infonce": ("cl_rows_kernel", "cl_table_kernel", "cl6_kernel", "cl6p_kernel", "cl_finalize_kernel",
                       "cl_table_reduce_kernel", "cl_table_reduce_nbwd_kernel")}
# launches of a class = launches of its primary kernels (one per gmr_* call)
PRIMARY = {"gemm": ("gemm_kernel", "gemm_glds_kernel"), "gemm_x6": ("gemm_x6_kernel",),
           "spmm": ("spmm_seg_kernel", "spmm_lane_kernel", "spmm_lane_jobs_kernel", "spmm_blk_kernel",
                    "spmm_chunk_kernel", "spmm_side_kernel",
                    "spmm_side_jobs_kernel"),
           "infonce": ("cl_rows_kernel", "cl6_rows")}
UTIL = {"gemm": ("gemm_kernel", "gemm_glds_kernel"), "gemm_x6": ("gemm_x6_kernel",), "spmm": (),
        "infonce": ("cl_rows_kernel", "cl_table_kernel", "cl6_kernel", "cl6p_kernel")}


def load(path, counter):
    out = []
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        base = name.split("<")[0]
        out.append((r.get("Dispatch_Id") or r.get("Correlation_Id"), base, float(r["Counter_Value"])))
        if base in ("cl6_kernel", "cl6p_kernel") and name.replace(" ", "").endswith(",false>"):
            out.append((None, "cl6_rows", 0.0))  # one split-bf16 InfoNCE call = one rows pass (marker)
    return out


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    mfma = load(sys.argv[3], "SQ_VALU_MFMA_BUSY_CYCLES")
    grbm = load(sys.argv[3], "GRBM_GUI_ACTIVE")
    with open(os.path.join(ROOT, "generative-multimodal-recommendation_amd", "gmr", "libgmr_hip.so"), "rb") as f:
        sha = hashlib.sha256(f.read()).hexdigest()
    res = {"lib_sha256": sha, "command": "GMR_SERIAL=1 python3 " + sys.argv[4],
           "source": "rocprofv3 --pmc, three passes: FETCH_SIZE | WRITE_SIZE | SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE",
           "correction": "bytes = 2 * FETCH_SIZE_KB * 1024 + WRITE_SIZE_KB * 1024 (gfx950 FETCH_SIZE halving)",
           "mfma_util": "sum SQ_VALU_MFMA_BUSY_CYCLES / (128 * sum GRBM_GUI_ACTIVE) over the class's primary kernels"}
    for cls, names in CLASSES.items():
        f = sum(v for _, n, v in fetch if n in names) * 1024 * 2
        w = sum(v for _, n, v in write if n in names) * 1024
        launches = sum(1 for _, n, _ in fetch if n in PRIMARY[cls])
        mb = sum(v for _, n, v in mfma if n in UTIL[cls])
        ga = sum(v for _, n, v in grbm if n in UTIL[cls])
        res[cls] = {"launches": launches, "fetch_bytes": f, "write_bytes": w,
                    "traffic_per_launch": (f + w) / max(launches, 1),
                    "mfma_busy_cycles": mb, "grbm_gui_active": ga,
                    "mfma_util": (mb / (128.0 * ga)) if ga > 0 and cls != "spmm" else None}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
