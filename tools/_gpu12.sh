set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_test_mode.py > gpurun_out/t14.log 2>&1 || { echo TESTFAIL; grep -E "^FAILED|^ERROR|Error" gpurun_out/t14.log | head; exit 1; }
tail -n 1 gpurun_out/t14.log
for rep in 1 2; do for lib in uni sload sload2; do
  echo "### $lib $rep"
  VR_LIB=$PWD/build_ab/$lib.so timeout -k 10 200 python tools/sweep.py --rounds 3 --configs t3e,t3,c3 > gpurun_out/ab14_$lib$rep.log 2>&1 || exit 1
  grep -E "median|digest" gpurun_out/ab14_$lib$rep.log
done; done
mkdir -p gpurun_out/lds
timeout -k 10 300 python3 tools/lds_pmc.py gpurun_out/lds/c3obl.json --camera oblique --extra-configs '' > gpurun_out/lds/c3obl.log 2>&1 || { echo LDSFAIL; tail -5 gpurun_out/lds/c3obl.log; exit 1; }
tail -n 1 gpurun_out/lds/c3obl.log
timeout -k 10 300 python3 tools/lds_pmc.py gpurun_out/lds/c3testo.json --mode test --camera oblique --extra-configs '' > gpurun_out/lds/c3testo.log 2>&1 || exit 1
tail -n 1 gpurun_out/lds/c3testo.log
timeout -k 10 300 python3 tools/lds_pmc.py gpurun_out/lds/c3test.json --mode test --extra-configs '' > gpurun_out/lds/c3test.log 2>&1 || exit 1
tail -n 1 gpurun_out/lds/c3test.log
