set -o pipefail
cd $GRAFT_REPO_ROOT
WL=r6_c3testo bash tools/r6_profiles.sh > gpurun_out/p18.log 2>&1 || { echo PROFFAIL; tail -5 gpurun_out/p18.log; exit 1; }
tail -2 gpurun_out/p18.log
python -c "import json;d=json.load(open('gpurun_out/prof_r6_c3testo/bench.json'));print('TEST oblique', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_mean'])"
timeout -k 10 300 python3 tools/lds_pmc.py gpurun_out/lds/c3testo_lin.json --mode test --camera oblique --extra-configs '' > gpurun_out/lds/c3testo_lin.log 2>&1 || exit 1
tail -n 1 gpurun_out/lds/c3testo_lin.log
