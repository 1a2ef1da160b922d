#!/bin/bash
# Height-field iteration loop: contact parity (kernel vs oracle and brute-force prisms), rough teacher
# forcing, then the C4 / C5 bench lines.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_physics.py -k "hfield" \
  > gpurun_out/hfq.log 2>&1 || { tail -30 gpurun_out/hfq.log; exit 1; }
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread "tests/test_gpu_teacher_forced.py::test_teacher_forced_step_parity[rough_dr]" \
  "tests/test_gpu_teacher_forced.py::test_teacher_forced_step_parity[rough_backlash_dr]" "tests/test_gpu_teacher_forced.py::test_teacher_forced_step_parity[rough_backlash_dr_autoreset]" > gpurun_out/hfq2.log 2>&1 || { tail -30 gpurun_out/hfq2.log; exit 1; }
tail -1 gpurun_out/hfq.log; tail -1 gpurun_out/hfq2.log
for C in C4 C5; do timeout -k 10 300 python bench.py --config $C --cpu-budget 0 > gpurun_out/bench_q_$C.json 2>/dev/null || exit 1; python -c "import json;d=json.load(open('gpurun_out/bench_q_$C.json'));print('$C', round(d['value']/1e6,3), 'M env-steps/s, kernel', round(d['roofline']['kernel_ms'],4), 'ms')"; done
