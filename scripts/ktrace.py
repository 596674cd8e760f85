"""Per-(kernel, grid) duration summary of a rocprofv3 kernel_trace.csv, in first-seen order.

python scripts/ktrace.py <kernel_trace.csv> [substring]
"""
import collections
import csv
import statistics
import sys


def main():
    path = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    od = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        if sub not in name:
            continue
        k = (name, r["Grid_Size_X"], r["VGPR_Count"], r["LDS_Block_Size"])
        od.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
    for (n, g, v, lds), ds in od.items():
        print(f"{n:40s} grid={g:>9s} vgpr={v:>4s} lds={lds:>6s} n={len(ds):4d} "
              f"median={statistics.median(ds):8.2f}us min={min(ds):8.2f}us")


if __name__ == "__main__":
    main()
