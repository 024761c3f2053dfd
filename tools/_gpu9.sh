set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
# VR_LIB=$PWD/build_ab/vlock.so timeout -k 10 900 python -u -m pytest --maxfail=25 -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_random.py tests/test_gpu_multi.py > gpurun_out/t9.log 2>&1 || { echo TESTFAIL; grep -E "^FAILED|^ERROR" gpurun_out/t9.log; exit 1; }
# tail -n 2 gpurun_out/t9.log
for rep in 1 2; do for lib in cur vlock; do
  echo "### $lib $rep"
  VR_LIB=$PWD/build_ab/$lib.so timeout -k 10 200 python tools/sweep.py --rounds 3 --configs c3,c4,c3s1,c2f > gpurun_out/ab9_$lib$rep.log 2>&1 || exit 1
  grep -E "median" gpurun_out/ab9_$lib$rep.log
  VR_LIB=$PWD/build_ab/$lib.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --extra 0 --cpu-baseline 0 --extra-configs '' > gpurun_out/b9_$lib$rep.json 2> gpurun_out/b9_$lib$rep.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/b9_$lib$rep.json'));print('bench C3 $lib', d['value'], d['ms_per_step'])"
done; done
