set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "cull or background or worklist or tile" > gpurun_out/t11.log 2>&1 || { echo TESTFAIL; grep -E "^FAILED|^ERROR|Error" gpurun_out/t11.log | head; exit 1; }
tail -n 1 gpurun_out/t11.log
for rep in 1 2; do for lib in cur bgv; do
  echo "### $lib $rep"
  VR_LIB=$PWD/build_ab/$lib.so timeout -k 10 200 python tools/sweep.py --rounds 3 --configs c3,c3s1,c3obl,t3e > gpurun_out/ab11_$lib$rep.log 2>&1 || exit 1
  grep -E "median" gpurun_out/ab11_$lib$rep.log
  VR_LIB=$PWD/build_ab/$lib.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --extra 0 --cpu-baseline 0 --extra-configs '' > gpurun_out/b11_$lib$rep.json 2> gpurun_out/b11_$lib$rep.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/b11_$lib$rep.json'));print('bench C3 $lib', d['value'], d['ms_per_step'])"
done; done
