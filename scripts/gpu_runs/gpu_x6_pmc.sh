#!/bin/bash
# SQ counters of the split-bf16 GEMM kernel (gemm_x6_kernel): MFMA busy, LDS bank conflicts / waits,
# one rocprofv3 --pmc pass per counter set, each under its own kill timeout.
set -o pipefail
TAG=${1:-x6pmc}
mkdir -p gpurun_out
export TMPDIR=/tmp
CMD="scripts/gemm_bench.py --only square8192,psample_out19k --tiles 256128 --mfma 6 --reps 3"
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d gpurun_out/${TAG}_a -o pmc -- python3 $CMD > gpurun_out/${TAG}_a.log 2>&1 || { echo "pass a failed"; tail -5 gpurun_out/${TAG}_a.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/${TAG}_b -o pmc -- python3 $CMD > gpurun_out/${TAG}_b.log 2>&1 || { echo "pass b failed"; tail -5 gpurun_out/${TAG}_b.log; exit 1; }
TAG_=$TAG python3 - <<'PY'
import csv, glob, collections, os
tag = os.environ["TAG_"]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for p in ("a", "b"):
    f = glob.glob(f"gpurun_out/{tag}_{p}/*counter_collection.csv")
    if not f: print("no csv", p); continue
    for r in csv.DictReader(open(f[0])):
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        if "gemm" not in n: continue
        agg[(n[:70], r.get("Grid_Size", ""))][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    mf = v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(1, 128 * v.get("GRBM_GUI_ACTIVE", 1))
    print(k, f"mfma_util={mf:.3f}", {c: f"{x:.3g}" for c, x in sorted(v.items())})
PY
