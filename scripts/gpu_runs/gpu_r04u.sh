#!/bin/bash
# r04u: InfoNCE A/B on one box (GMR_CL_PIPE x GMR_CL_FIXUP; contrast_bench at the DiffMM baby shapes) + the
# kernel split of the default; the DiffMM epoch with the fixup on / off; GenRecV1 with 256-deep split-K slabs.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for p in 1 0; do for f in 1 0; do
  echo "[GMR_CL_PIPE=$p GMR_CL_FIXUP=$f]"
  GMR_CL_PIPE=$p GMR_CL_FIXUP=$f timeout -k 10 120 python scripts/contrast_bench.py --reps 30 2>&1 | grep -v amdgpu.ids || exit 1
done; done > gpurun_out/r04u_contrast_ab.txt
cat gpurun_out/r04u_contrast_ab.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04u_prof -o run -- python scripts/contrast_bench.py --reps 30 > gpurun_out/r04u_prof.log 2>&1 || { tail -20 gpurun_out/r04u_prof.log; exit 1; }
f=$(find gpurun_out/r04u_prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r04u_contrast_kernel_stats.csv; cut -d, -f1-4 gpurun_out/r04u_contrast_kernel_stats.csv | cut -c1-150 | head -8
B="python bench.py --model diffmm --no-legs --steps 5 --warmup 2 --no-cpu-baseline --no-probe"
for f in 1 0; do
  GMR_CL_FIXUP=$f timeout -k 10 300 $B > gpurun_out/r04u_diffmm_fix$f.json 2> gpurun_out/r04u_diffmm_fix$f.err || { tail -20 gpurun_out/r04u_diffmm_fix$f.err; exit 1; }
  echo "fixup=$f $(cut -c1-220 gpurun_out/r04u_diffmm_fix$f.json)"; grep "phases" gpurun_out/r04u_diffmm_fix$f.err | tail -2
done
G="python bench.py --model genrecv1 --steps 3 --warmup 1 --no-cpu-baseline --no-probe"
for s in 512 256; do
  GMR_X6_MIN_SLAB=$s timeout -k 10 300 $G > gpurun_out/r04u_genrec_slab$s.json 2> gpurun_out/r04u_genrec_slab$s.err || { tail -20 gpurun_out/r04u_genrec_slab$s.err; exit 1; }
  echo "slab=$s $(cut -c1-220 gpurun_out/r04u_genrec_slab$s.json)"
done
