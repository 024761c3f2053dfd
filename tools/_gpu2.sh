set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do for lib in pt k8; do
  echo "### $lib $rep"
  VR_LIB=$PWD/build_ab/$lib.so timeout -k 10 200 python tools/sweep.py --rounds 3 --configs t3eo,t3so,t3e --variants "test_corners=3;test_corners=0" > gpurun_out/ab2_$lib$rep.log 2>&1 || exit 1
  grep -E "median" gpurun_out/ab2_$lib$rep.log
done; done
for rep in 1 2; do
timeout -k 10 300 python bench.py --mode test --camera oblique --steps 20 --warmup 5 --extra 0 --cpu-baseline 0 --extra-configs '' > gpurun_out/b_testo$rep.json 2> gpurun_out/b_testo$rep.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/b_testo$rep.json'));print('bench test oblique', d['value'], d['ms_per_step'])"
timeout -k 10 300 python bench.py --mode test --steps 20 --warmup 5 --extra 0 --cpu-baseline 0 --extra-configs '' > gpurun_out/b_test$rep.json 2> gpurun_out/b_test$rep.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/b_test$rep.json'));print('bench test default', d['value'], d['ms_per_step'])"
done
