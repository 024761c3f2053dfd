set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/lds
for rep in 1 2; do for lib in cur w6; do
  echo "### $lib $rep"
  VR_LIB=$PWD/build_ab/$lib.so timeout -k 10 200 python tools/sweep.py --rounds 3 --configs t3eo,t3ro > gpurun_out/ab18_$lib$rep.log 2>&1 || exit 1
  grep -E "median" gpurun_out/ab18_$lib$rep.log
done; done
timeout -k 10 300 python3 tools/lds_pmc.py gpurun_out/lds/c3testo_lin.json --mode test --camera oblique --extra-configs '' > gpurun_out/lds/c3testo_lin.log 2>&1 || exit 1
tail -n 1 gpurun_out/lds/c3testo_lin.log
