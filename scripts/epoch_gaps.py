"""Idle time of whole epochs from a rocprofv3 kernel trace taken with the side streams on (the timed
configuration): the union of kernel intervals per epoch (GPU busy), the idle remainder, and the largest
idle gaps with the kernels on either side (host stalls: synchronisations, host-side planning, launch
gaps).  Epochs are cut at the diffusion phase's first denoiser launch after each BPR phase.

python scripts/epoch_gaps.py <kernel_trace.csv[.gz]> [--top 25] [--min-us 20]
"""
import argparse
import csv
import gzip


def load(path):
    op = gzip.open if path.endswith(".gz") else open
    rows = []
    with op(path, "rt") as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name[:60]))
    rows.sort()
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--min-us", type=float, default=20.0)
    a = ap.parse_args()
    rows = load(a.trace)
    # epoch starts: an adam step of the rec phase followed by a diffusion-phase kernel marks the boundary;
    # simplest robust cut: the first qsample kernel after a bpr kernel
    starts, seen_bpr = [], True
    for i, (_, _, n) in enumerate(rows):
        if "bpr_kernel" in n:
            seen_bpr = True
        elif "qsample" in n and seen_bpr:
            starts.append(i)
            seen_bpr = False
    starts.append(len(rows))
    print(f"{len(rows)} kernels, {len(starts) - 1} epochs (cut at the diffusion phase's first q_sample)")
    gaps_all = []
    for e in range(len(starts) - 1):
        seg = rows[starts[e]:starts[e + 1]]
        t0, t1 = seg[0][0], max(r[1] for r in seg)
        busy, cur_s, cur_e, prev = 0, seg[0][0], seg[0][1], seg[0]
        for s, en, n in seg[1:]:
            if s > cur_e:
                busy += cur_e - cur_s
                gaps_all.append((s - cur_e, e, prev[2], n))
                cur_s, cur_e = s, en
            else:
                cur_e = max(cur_e, en)
            if en >= cur_e:
                prev = (s, en, n)
        busy += cur_e - cur_s
        wall = t1 - t0
        print(f"epoch {e}: wall {wall / 1e6:.2f} ms, GPU busy {busy / 1e6:.2f} ms ({busy / wall:.3f}), "
              f"idle {(wall - busy) / 1e6:.2f} ms, {len(seg)} kernels")
    gaps_all.sort(reverse=True)
    print(f"largest idle gaps (>= {a.min_us} us):")
    for g, e, before, after in gaps_all[:a.top]:
        if g / 1e3 < a.min_us:
            break
        print(f"  {g / 1e3:9.1f} us  epoch {e}  after {before:<45} before {after}")
    tot = sum(g for g, *_ in gaps_all if g / 1e3 >= a.min_us)
    print(f"sum of gaps >= {a.min_us} us: {tot / 1e6:.2f} ms over {len(starts) - 1} epochs")


if __name__ == "__main__":
    main()
