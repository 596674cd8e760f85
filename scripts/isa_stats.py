"""Per-kernel ISA statistics from a hipcc --save-temps gfx950 .s file.

python scripts/isa_stats.py <file.s> <kernel-name-substring>
Prints MFMA / global_load_lds / s_waitcnt vmcnt(0) / barrier counts and the register, scratch and
LDS figures of every matching kernel.
"""
import re
import sys


def main():
    path, pat = sys.argv[1], sys.argv[2]
    s = open(path).read()
    for m in re.finditer(r'^(_Z\S*' + re.escape(pat) + r'\S*):', s, re.M):
        name = m.group(1)
        end = s.index('.Lfunc_end', m.end())
        body = s[m.end():end]
        i = s.find('.amdhsa_kernel ' + name)
        md = s[i:i + 4000]

        def g(k):
            r = re.search(r'\.amdhsa_' + k + r' (\d+)', md)
            return r.group(1) if r else "?"
        print(f"{name[:90]}\n   mfma {body.count('v_mfma')} glds {body.count('global_load_lds')} "
              f"vmcnt(0) {len(re.findall(r'vmcnt[(]0[)]', body))} barrier {body.count('s_barrier')} "
              f"vgpr {g('next_free_vgpr')} accum_offset {g('accum_offset')} scratch {g('private_segment_fixed_size')} "
              f"lds {g('group_segment_fixed_size')}")


if __name__ == "__main__":
    main()
