# The -m gpu suite (run through gpurun), one process, per-test timeout; log under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread "$@" > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "PASS|FAIL|Error|error" gpurun_out/gpu_tests.log | tail -30; exit 1; }
grep -cE "PASSED" gpurun_out/gpu_tests.log; tail -1 gpurun_out/gpu_tests.log
