set -o pipefail
mkdir -p gpurun_out
for nx in 1024 2048 4096; do
  timeout -k 10 200 python tools/tb_sweep.py --nx $nx --n 8192 --interior --depths 8 --variants 23,16407,2071 --waves 0,1024,2048,3072 --rounds 5 --iters 200 --json gpurun_out/sweep_r2_bperm_$nx.jsonl > gpurun_out/sweep_r2_bperm_$nx.txt 2>&1 || exit 1
  cat gpurun_out/sweep_r2_bperm_$nx.txt
done
