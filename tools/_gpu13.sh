set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_test_mode.py > gpurun_out/t15.log 2>&1 || { echo TESTFAIL; grep -E "^FAILED|^ERROR|Error" gpurun_out/t15.log | head; exit 1; }
tail -n 1 gpurun_out/t15.log
for rep in 1 2; do for lib in k8 k4 k16; do
  echo "### $lib $rep"
  VR_LIB=$PWD/build_ab/$lib.so timeout -k 10 200 python tools/sweep.py --rounds 3 --configs t3e,t3,t3s,t3x > gpurun_out/ab15_$lib$rep.log 2>&1 || exit 1
  grep -E "median" gpurun_out/ab15_$lib$rep.log
done; done
