set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/final
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/t23.log 2>&1 || { echo TESTFAIL; grep -E "^FAILED|^ERROR|Error|assert" gpurun_out/t23.log | head -20; exit 1; }
tail -n 1 gpurun_out/t23.log
timeout -k 10 200 python tools/sweep.py --rounds 3 --configs t3e,t3s,t3x,c3 > gpurun_out/ab23.log 2>&1 || exit 1
grep -E "median" gpurun_out/ab23.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final/smoke.log 2>&1 || { echo SMOKEFAIL; exit 1; }
tail -n 1 gpurun_out/final/smoke.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err || { echo BENCHFAIL; tail gpurun_out/final/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/final/bench.json'));print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'])"
