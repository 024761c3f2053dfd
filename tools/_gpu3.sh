set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do for lib in cur pf; do
  VR_LIB=$PWD/build_ab/$lib.so timeout -k 10 300 python bench.py --volume c5 --width 3840 --height 2160 --samples 4096 --steps 20 --warmup 5 --extra 0 --cpu-baseline 0 --extra-configs '' > gpurun_out/c5_$lib$rep.json 2> gpurun_out/c5_$lib$rep.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/c5_$lib$rep.json'));print('C5 $lib', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_mean'])"
done; done
for rep in 1 2; do for lib in cur w6; do
  echo "### $lib $rep"
  VR_LIB=$PWD/build_ab/$lib.so timeout -k 10 200 python tools/sweep.py --rounds 3 --configs t3eo,t3so --variants "test_corners=0" > gpurun_out/ab3_$lib$rep.log 2>&1 || exit 1
  grep -E "median" gpurun_out/ab3_$lib$rep.log
done; done
