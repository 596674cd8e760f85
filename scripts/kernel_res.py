"""VGPR / AGPR / scratch / LDS of the kernels in a hipcc -save-temps .s file (filter by substring).

python scripts/kernel_res.py build/x.s [substring]
"""
import re
import sys

s = open(sys.argv[1]).read()
flt = sys.argv[2] if len(sys.argv) > 2 else ""
for blk in s.split(".end_amdhsa_kernel"):
    m = re.search(r"\.amdhsa_kernel (\S+)", blk)
    if not m or flt not in m.group(1):
        continue
    g = lambda k: (re.search(r"\.amdhsa_%s (\d+)" % k, blk) or [None, "?"])[1]  # noqa: E731
    print(f"{m.group(1)[-70:]:72s} vgpr {g('next_free_vgpr'):>4s} accoff {g('accum_offset'):>4s} "
          f"scratch {g('private_segment_fixed_size'):>4s} lds {g('group_segment_fixed_size'):>6s}")
