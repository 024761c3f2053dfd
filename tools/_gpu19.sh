set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/t20.log 2>&1 || { echo TESTFAIL; grep -E "^FAILED|^ERROR|Error|assert" gpurun_out/t20.log | head -20; exit 1; }
tail -n 1 gpurun_out/t20.log
timeout -k 10 200 python tools/sweep.py --rounds 3 --configs t3eo,t3ro,t3e,c3 > gpurun_out/ab20.log 2>&1 || exit 1
grep -E "median" gpurun_out/ab20.log
