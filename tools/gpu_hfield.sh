#!/bin/bash
# Height-field parity on the GPU: prism contacts vs the oracle, rough physics, rough teacher forcing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -s \
  "tests/test_gpu_physics.py::test_hfield_prism_contacts_match_oracle" \
  "tests/test_gpu_physics.py::test_forward_parity" "tests/test_gpu_physics.py::test_substep_parity" \
  "tests/test_gpu_teacher_forced.py::test_teacher_forced_step_parity[rough_dr]" \
  "tests/test_gpu_teacher_forced.py::test_teacher_forced_step_parity[rough_backlash_dr]" \
  "tests/test_gpu_teacher_forced.py::test_teacher_forced_step_parity[rough_backlash_dr_autoreset]" \
  > gpurun_out/hfield_tests.log 2>&1
rc=$?
tail -30 gpurun_out/hfield_tests.log
exit $rc
