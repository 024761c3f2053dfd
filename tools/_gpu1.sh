set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_test_mode.py tests/test_gpu_bench.py::test_peer_traffic_fields_two_part_group tests/test_gpu_parity.py::test_point_cloud_colours_on_the_screenshot_hull > gpurun_out/t_testmode.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/t_testmode.log; exit 1; }
tail -3 gpurun_out/t_testmode.log
for rep in 1 2; do for lib in base pt axdeal; do
  echo "### $lib $rep"
  VR_LIB=$PWD/build_ab/$lib.so timeout -k 10 200 python tools/sweep.py --rounds 3 --configs ${CFGS:-t3eo,t3e,t3xo,t3x} > gpurun_out/ab_$lib$rep.log 2>&1 || exit 1
  grep -E "median|digest" gpurun_out/ab_$lib$rep.log
done; done
