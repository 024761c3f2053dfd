set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do for lib in ax1 ax7; do
  echo "### $lib $rep"
  VR_LIB=$PWD/build_ab/$lib.so timeout -k 10 200 python tools/sweep.py --rounds 3 --configs t3e,t3,t3s,t3x > gpurun_out/ab22_$lib$rep.log 2>&1 || exit 1
  grep -E "median" gpurun_out/ab22_$lib$rep.log
done; done
