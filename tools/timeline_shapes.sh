set -o pipefail
for args in ${TL_ARGS:-"--depth 12" "--depth 8" "--nx 1024 --depth 8 --interior" "--nx 2048 --depth 8 --interior" "--nx 4096 --depth 12 --interior"}; do
  timeout -k 5 120 python tools/wave_timeline.py $args >> gpurun_out/timeline.jsonl 2>gpurun_out/timeline.err || exit 1
done
cat gpurun_out/timeline.jsonl
