# Depthwise conv images in flight (k = 7, M shape).  Measured with alternate libraries built from
# norm_dw.hip with launch_dw3's PF = 1 / 2 / 3 / 4 (two interleaved passes each):
#   alone (tools/kern_bench.py --only dw): 53.4 / 51.2-51.5 / 54.4 / 55.2 us
#   M forward: 10,201 10,224 / 10,254 10,231 10,271 10,242 / 10,230 10,212 10,211 10,198 / 10,190 10,191 img/s
# PF = 2 is the default since.  This script re-checks the default build: tests, kernel time, M step.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_model.py -k "dwconv or model" > gpurun_out/r4_pf_tests.log 2>&1 || { tail -30 gpurun_out/r4_pf_tests.log; exit 1; }
tail -1 gpurun_out/r4_pf_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_pf_smoke.log 2>&1 || { tail -20 gpurun_out/r4_pf_smoke.log; exit 1; }
grep smoke: gpurun_out/r4_pf_smoke.log
timeout -k 10 200 python tools/kern_bench.py --only dw > gpurun_out/r4_pf_kb.log 2>&1 && grep 'dwconv_ln k3' gpurun_out/r4_pf_kb.log
timeout -k 10 300 python bench.py > gpurun_out/r4_pf_m.log 2>&1 || { tail -20 gpurun_out/r4_pf_m.log; exit 1; }
tail -n 1 gpurun_out/r4_pf_m.log | cut -c1-400
