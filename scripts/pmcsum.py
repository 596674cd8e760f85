"""Median counter values per (kernel, grid) from rocprofv3 --pmc counter_collection.csv files.

python scripts/pmcsum.py <csv> [<csv> ...] [--filter substring]
"""
import collections
import csv
import statistics
import sys


def main():
    args = sys.argv[1:]
    sub = ""
    if "--filter" in args:
        i = args.index("--filter")
        sub = args[i + 1]
        args = args[:i] + args[i + 2:]
    od = collections.OrderedDict()
    for f in args:
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
            if sub not in name:
                continue
            k = (name, r["Grid_Size"])
            od.setdefault(k, collections.OrderedDict()).setdefault(r["Counter_Name"], []).append(
                float(r["Counter_Value"]))
    for (n, g), cs in od.items():
        print(f"{n} grid={g}: " + ", ".join(f"{c}={statistics.median(v):.0f}" for c, v in cs.items()))


if __name__ == "__main__":
    main()
