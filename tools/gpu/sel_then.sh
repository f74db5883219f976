# selected GPU tests ($1, quoted pytest selector), then the script $2 (if the tests passed)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest $1 -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_sel.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_sel.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error|Timeout" gpurun_out/pytest_sel.log | head -30; exit 1; fi
[ -n "$2" ] && bash $2
