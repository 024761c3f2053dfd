C5="--volume c5 --width 3840 --height 2160 --samples 4096 --steps 20 --warmup 3 --cpu-baseline 0 --extra 0 --traffic-json /nonexistent"
args=()
for rep in 1 2; do
for v in win0 win1; do
 args+=("200|c5x_${v}_$rep|VR_LIB=\$PWD/build_ab/$v.so python bench.py $C5 --flags exact")
 args+=("200|c5e_${v}_$rep|VR_LIB=\$PWD/build_ab/$v.so python bench.py $C5")
done
done
args+=("700|gputests|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread")
args+=("300|bench|python3 bench.py --gpus 1 --steps 20 --warmup 5")
tools/gpu_session.sh "${args[@]}"
