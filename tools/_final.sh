set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/final
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/final/gpu_tests.log 2>&1 || { echo TESTFAIL; grep -E "^FAILED|^ERROR|Error" gpurun_out/final/gpu_tests.log | head; exit 1; }
tail -n 1 gpurun_out/final/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final/smoke.log 2>&1 || { echo SMOKEFAIL; tail gpurun_out/final/smoke.log; exit 1; }
tail -n 1 gpurun_out/final/smoke.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err || { echo BENCHFAIL; tail gpurun_out/final/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/final/bench.json'));print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline']['value'])"
