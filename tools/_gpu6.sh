set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
C5="--volume c5 --width 3840 --height 2160 --samples 4096 --steps 20 --warmup 5 --extra-configs ''"
for rep in 1 2; do for lib in cur rw6; do
  VR_LIB=$PWD/build_ab/$lib.so timeout -k 10 300 python bench.py --volume c5 --width 3840 --height 2160 --samples 4096 --steps 20 --warmup 5 --extra 0 --cpu-baseline 0 --extra-configs '' > gpurun_out/c5w_$lib$rep.json 2> gpurun_out/c5w_$lib$rep.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/c5w_$lib$rep.json'));print('C5 $lib', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_mean'])"
done; done
timeout -k 10 1000 bash tools/round_profile.sh r6_c5 --volume c5 --width 3840 --height 2160 --samples 4096 --steps 20 --warmup 5 --extra-configs '' || exit 1
VR_LIB=$PWD/build_ab/pf.so timeout -k 10 1000 bash tools/round_profile.sh r6_c5pf --volume c5 --width 3840 --height 2160 --samples 4096 --steps 20 --warmup 5 --extra-configs '' || exit 1
for t in r6_c5 r6_c5pf; do python -c "import json;d=json.load(open('gpurun_out/prof_$t/traffic.json'));print('$t', {k:int(v) for k,v in d['sq'].items()}, d['sq_split'], d['hbm_read_bytes_corrected'], d['cache'])"; done
