set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/tb_sweep.py --nx 1024 --n 8192 --interior --depths 8 --variants 23,4119,1047,5143 --waves 1024,2048 --rounds 5 --iters 200 --json gpurun_out/sweep_r2_diag_1024.jsonl > gpurun_out/sweep_r2_diag_1024.txt 2>&1 || exit 1
cat gpurun_out/sweep_r2_diag_1024.txt
timeout -k 10 200 python tools/tb_sweep.py --nx 8192 --n 8192 --depths 12 --variants 2071,6167,3095,7191 --waves 0 --rounds 5 --iters 240 --json gpurun_out/sweep_r2_diag_8192.jsonl > gpurun_out/sweep_r2_diag_8192.txt 2>&1 || exit 1
cat gpurun_out/sweep_r2_diag_8192.txt
