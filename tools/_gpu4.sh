set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/t_all.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/t_all.log; exit 1; }
tail -3 gpurun_out/t_all.log
for rep in 1 2; do for lib in cur m24; do
  echo "### $lib $rep"
  VR_LIB=$PWD/build_ab/$lib.so timeout -k 10 200 python tools/sweep.py --rounds 3 --configs t3eo,t3so,t3xo > gpurun_out/ab4_$lib$rep.log 2>&1 || exit 1
  grep -E "median" gpurun_out/ab4_$lib$rep.log
done; done
timeout -k 10 1000 bash tools/round_profile.sh r6_c3testo --steps 20 --warmup 5 --mode test --camera oblique --extra-configs '' || exit 1
python -c "import json;d=json.load(open('gpurun_out/prof_r6_c3testo/traffic.json'));print(d['sq'], d['sq_split'], d['hbm_read_bytes_corrected'])"; python -c "import json;d=json.load(open('gpurun_out/prof_r6_c3testo/bench.json'));print(d['value'], d['ms_per_step'], d['roofline']['samples_evaluated'], d['roofline']['kernel_ms_mean'])"
