#!/bin/bash
# r04i: class plan (degree <= 16) with counted vmcnt waits (unconditional loads, compile-time beta): probe, SpMM kernel
# tests (both plan forms), then the DiffMM phase / baby parity tests on the new default.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python scripts/micro/dump_graph.py baby norm_adj /tmp/na.bin > gpurun_out/r04i_probe.txt || exit 1
python scripts/micro/dump_graph.py baby ui_top1 /tmp/ui.bin >> gpurun_out/r04i_probe.txt || exit 1
timeout -k 10 240 scripts/micro/side_iso /tmp/na.bin >> gpurun_out/r04i_probe.txt 2>&1 || { tail -20 gpurun_out/r04i_probe.txt; exit 1; }
timeout -k 10 240 scripts/micro/side_iso /tmp/ui.bin >> gpurun_out/r04i_probe.txt 2>&1 || { tail -20 gpurun_out/r04i_probe.txt; exit 1; }
grep -E 'full|user side only|item side only|classes|T=' gpurun_out/r04i_probe.txt | head -120
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -k "spmm" > gpurun_out/r04i_spmm_tests.log 2>&1 || { tail -30 gpurun_out/r04i_spmm_tests.log; exit 1; }
tail -3 gpurun_out/r04i_spmm_tests.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 420 --timeout-method thread -p no:cacheprovider \
  tests/test_diffmm_gpu.py tests/test_phases_gpu.py tests/test_baby_gpu.py tests/test_sports_gpu.py > gpurun_out/r04i_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r04i_tests.log
exit $rc
