"""GPU busy fraction of the BPR/contrastive phase from a rocprofv3 kernel trace (no --stats needed).

python scripts/trace_gaps.py <kernel_trace.csv> [--steps 20]
Takes the last `steps` rec steps (each ends with its Adam launch after a bpr_kernel), and reports
wall time per step, the union of kernel intervals (GPU busy), the idle gaps, and per-kernel totals.
"""
import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name[:70], r.get("Queue_Id", "")))
    rows.sort()
    bpr = [i for i, r in enumerate(rows) if "bpr_kernel" in r[2] or "bpr_sqnorm_kernel" in r[2]]
    # step k = from its bpr_kernel back to the previous step's adam_kernel (exclusive)
    adam = [i for i, r in enumerate(rows) if "adam_kernel" in r[2] or "adam4_kernel" in r[2]]
    ends = []
    for b in bpr:
        nxt = [j for j in adam if j > b]
        if nxt:
            ends.append(nxt[0])
    ends = sorted(set(ends))[-(a.steps + 1):]
    lo, hi = ends[0] + 1, ends[-1]
    win = rows[lo:hi + 1]
    t0, t1 = win[0][0], max(r[1] for r in win)
    busy, cur_s, cur_e = 0, None, None
    gaps = []
    for s, e, _, _ in win:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    n = len(ends) - 1
    tot = defaultdict(float)
    cnt = defaultdict(int)
    for s, e, name, _ in win:
        tot[name] += e - s
        cnt[name] += 1
    print(f"{n} steps, {len(win)} kernels ({len(win) / n:.1f}/step): wall {(t1 - t0) / 1e3 / n:.1f} us/step, "
          f"GPU busy (union) {busy / 1e3 / n:.1f} us/step = {busy / (t1 - t0):.3f}, "
          f"sum of kernel durations {sum(tot.values()) / 1e3 / n:.1f} us/step")
    gaps.sort()
    if gaps:
        print(f"idle gaps: {len(gaps) / n:.1f}/step, total {sum(gaps) / 1e3 / n:.1f} us/step, "
              f"median {gaps[len(gaps) // 2] / 1e3:.1f} us, p90 {gaps[int(len(gaps) * 0.9)] / 1e3:.1f} us, "
              f"max {gaps[-1] / 1e3:.1f} us")
    for name, v in sorted(tot.items(), key=lambda kv: -kv[1])[:30]:
        print(f"  {v / 1e3 / n:8.1f} us/step  {cnt[name] / n:5.1f}/step  {name}")


if __name__ == "__main__":
    main()
