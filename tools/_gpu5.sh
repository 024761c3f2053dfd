set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6_scale
timeout -k 10 400 python tools/scale_probe.py > gpurun_out/r6_scale/probe.json 2> gpurun_out/r6_scale/probe.err || { tail -20 gpurun_out/r6_scale/probe.err; exit 1; }
cat gpurun_out/r6_scale/probe.json
for rep in 1 2; do for lib in m24 uni sel; do
  echo "### $lib $rep"
  VR_LIB=$PWD/build_ab/$lib.so timeout -k 10 200 python tools/sweep.py --rounds 3 --configs t3eo,t3so,t3xo > gpurun_out/ab5_$lib$rep.log 2>&1 || exit 1
  grep -E "median|digest" gpurun_out/ab5_$lib$rep.log
done; done
