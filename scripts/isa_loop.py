"""Print the compressed instruction stream of one kernel of a hipcc -save-temps .s file.

python scripts/isa_loop.py file.s <kernel substring> [max lines]
Runs of the same opcode are folded into 'op xN'; labels, branches and waits are kept verbatim.
"""
import sys

lines = open(sys.argv[1]).read().split("\n")
key = sys.argv[2]
lim = int(sys.argv[3]) if len(sys.argv) > 3 else 400
start = next(i for i, l in enumerate(lines) if key in l and l.split(";")[0].strip().endswith(":") and not l.startswith("\t"))
out = []
for l in lines[start + 1:]:
    t = l.split(";")[0].strip()
    if t.startswith(".Lfunc_end"):
        break
    if not t or t.startswith("."):
        if t.startswith(".LBB"):
            out.append(t)
        continue
    op = t.split()[0]
    if op.startswith(("s_waitcnt", "s_cbranch", "s_barrier", "s_branch", "s_setprio", "s_sched")):
        out.append(t)
    else:
        out.append(op)
comp, prev, n = [], None, 0
for o in out:
    if o == prev:
        n += 1
        continue
    if prev is not None:
        comp.append(f"{prev} x{n}" if n > 1 else prev)
    prev, n = o, 1
comp.append(f"{prev} x{n}" if n > 1 else prev)
print("\n".join(comp[:lim]))
