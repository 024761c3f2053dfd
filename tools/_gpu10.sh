set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do for lib in cur lazy; do
  echo "### $lib $rep"
  VR_LIB=$PWD/build_ab/$lib.so timeout -k 10 200 python tools/sweep.py --rounds 3 --configs t3eo,t3e > gpurun_out/ab10_$lib$rep.log 2>&1 || exit 1
  grep -E "median" gpurun_out/ab10_$lib$rep.log
done; done
