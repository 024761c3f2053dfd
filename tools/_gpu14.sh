set -o pipefail
cd $GRAFT_REPO_ROOT
WL=r6_c3test bash tools/r6_profiles.sh > gpurun_out/p16.log 2>&1 || { echo PROFFAIL; tail -5 gpurun_out/p16.log; exit 1; }
tail -3 gpurun_out/p16.log
python -c "import json;d=json.load(open('gpurun_out/prof_r6_c3test/bench.json'));print('TEST default', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_mean'])"
