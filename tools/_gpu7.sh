set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_test_mode.py tests/test_gpu_parity.py tests/test_gpu_random.py > gpurun_out/t_7.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/t_7.log; exit 1; }
tail -2 gpurun_out/t_7.log
for rep in 1 2; do for lib in cur fd; do
  echo "### $lib $rep"
  VR_LIB=$PWD/build_ab/$lib.so timeout -k 10 200 python tools/sweep.py --rounds 3 --configs t3eo,t3so,t3xo > gpurun_out/ab7_$lib$rep.log 2>&1 || exit 1
  grep -E "median" gpurun_out/ab7_$lib$rep.log
done; done
for rep in 1 2; do
timeout -k 10 300 python bench.py --mode test --camera oblique --steps 20 --warmup 5 --extra 0 --cpu-baseline 0 --extra-configs '' > gpurun_out/b7_testo$rep.json 2> gpurun_out/b7_testo$rep.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/b7_testo$rep.json'));print('bench test oblique', d['value'], d['ms_per_step'])"
done
