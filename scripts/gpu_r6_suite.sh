#!/bin/bash
# Full GPU suite + smoke (the driver's round-end gate), logs under gpurun_out/r6_suite.
mkdir -p gpurun_out/r6_suite
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r6_suite/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r6_suite/pytest.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|Error" gpurun_out/r6_suite/pytest.log | head -20; exit $rc; fi
timeout -k 10 400 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6_suite/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/r6_suite/smoke.log; exit $rc
