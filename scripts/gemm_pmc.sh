#!/bin/bash
# SQ counters of the GEMM kernel on two shapes (LDS bank conflicts, LDS waits, MFMA busy): one
# rocprofv3 --pmc pass per counter set, each under its own kill timeout.
set -o pipefail
TAG=${1:-gemmpmc}
mkdir -p gpurun_out
export TMPDIR=/tmp
CMD="scripts/gemm_bench.py --only psample_h19k,square8192,train_out --tiles 128,256 --reps 3"
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d gpurun_out/${TAG}_a -o pmc -- python3 $CMD > gpurun_out/${TAG}_a.log 2>&1 || { echo "pass a failed"; tail -5 gpurun_out/${TAG}_a.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAVES --output-format csv -d gpurun_out/${TAG}_b -o pmc -- python3 $CMD > gpurun_out/${TAG}_b.log 2>&1 || { echo "pass b failed"; tail -5 gpurun_out/${TAG}_b.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections, os
tag = os.environ.get("TAG_", "gemmpmc")
for p in ("a", "b"):
    f = glob.glob(f"gpurun_out/{tag}_{p}/*counter_collection.csv")
    if not f: print("no csv", p); continue
    agg = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
    for r in csv.DictReader(open(f[0])):
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        if "gemm" not in n: continue
        key = (n[:60], r.get("Grid_Size", ""))
        agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, v in agg.items():
        print(p, k, {c: f"{x:.3g}" for c, x in v.items()})
PY
