set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do for lib in gw1 gw7; do
  echo "### $lib $rep"
  VR_LIB=$PWD/build_ab/$lib.so timeout -k 10 200 python tools/sweep.py --rounds 3 --configs c3obl,c3obls,c3con,c3 > gpurun_out/ab16_$lib$rep.log 2>&1 || exit 1
  grep -E "median" gpurun_out/ab16_$lib$rep.log
done; done
