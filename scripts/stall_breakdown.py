"""Per-kernel stall / LDS breakdown from the two SQ passes of scripts/gpu_runs/gpu_r06s.sh (same counters as
round 5's gpu_r05zy.sh).

python scripts/stall_breakdown.py gpurun_out/r06s_a/pmc_counter_collection.csv gpurun_out/r06s_b/pmc_counter_collection.csv

Fractions of SQ_WAVE_CYCLES: park = SQ_WAIT_ANY (s_waitcnt / barrier), stall = SQ_WAIT_INST_ANY (issue stall: MFMA
RAW / pipe busy), issue = SQ_ACTIVE_INST_ANY; ldsconf = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE; mfmaU =
SQ_VALU_MFMA_BUSY_CYCLES / (128 GRBM_GUI_ACTIVE) over the kernel's dispatches; valu/mfma = SQ_INSTS_VALU /
SQ_INSTS_MFMA.  Kernels ordered by their share of all wave cycles.
"""
import collections
import csv
import sys


def load(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:58]
        agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
    return agg


def main():
    a, b = load(sys.argv[1]), load(sys.argv[2])
    total = sum(v["SQ_WAVE_CYCLES"] for v in a.values()) or 1.0
    print(f"{'kernel':58s} {'wave%':>6s} {'park':>5s} {'stall':>5s} {'issue':>5s} {'ldsconf':>7s} {'mfmaU':>6s} "
          f"{'valu/mfma':>9s}")
    for name, v in sorted(a.items(), key=lambda kv: -kv[1]["SQ_WAVE_CYCLES"])[:24]:
        w = v["SQ_WAVE_CYCLES"] or 1.0
        bb = b.get(name, {})
        lds = bb.get("SQ_LDS_IDX_ACTIVE", 0.0)
        conf = bb.get("SQ_LDS_BANK_CONFLICT", 0.0) / lds if lds else 0.0
        grbm = bb.get("GRBM_GUI_ACTIVE", 0.0)
        mfu = bb.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (128 * grbm) if grbm else 0.0
        nm = bb.get("SQ_INSTS_MFMA", 0.0)
        vm = bb.get("SQ_INSTS_VALU", 0.0) / nm if nm else float("nan")
        print(f"{name:58s} {100 * w / total:6.1f} {v['SQ_WAIT_ANY'] / w:5.2f} {v['SQ_WAIT_INST_ANY'] / w:5.2f} "
              f"{v['SQ_ACTIVE_INST_ANY'] / w:5.2f} {conf:7.3f} {mfu:6.2f} {vm:9.2f}")


if __name__ == "__main__":
    main()
