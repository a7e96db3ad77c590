#!/bin/bash
# Round 4: k_policy<2> from 20 480 to 32 768 rows (was <1> / <4>): every GPU
# test, then the default policy pass timing at 24 576 / 32 768 / 65 536 rows.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
mkdir -p gpurun_out/mtr
export PYTHONUNBUFFERED=1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/mtr/pytest.log 2>&1
rc=$?; echo "tests: $(tail -n 1 gpurun_out/mtr/pytest.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/mtr/pytest.log; exit $rc; }
for W in 24576 32768 65536; do
    timeout -k 10 120 python3 tools/policy_time.py --worlds $W 2>&1 | grep -v amdgpu.ids | sed "s|^|default |" || exit 1
done
