set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for lib in lock locknm; do
VR_LIB=$PWD/build_ab/$lib.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_test_mode.py > gpurun_out/t8_$lib.log 2>&1 || { echo TESTFAIL $lib; tail -30 gpurun_out/t8_$lib.log; }
tail -1 gpurun_out/t8_$lib.log
done
for rep in 1 2; do for lib in cur lock locknm; do
  echo "### $lib $rep"
  VR_LIB=$PWD/build_ab/$lib.so timeout -k 10 200 python tools/sweep.py --rounds 3 --configs t3e,t3s,t3x,t3 > gpurun_out/ab8_$lib$rep.log 2>&1 || exit 1
  grep -E "median|digest" gpurun_out/ab8_$lib$rep.log
done; done
