set -e
O=gpurun_out/da; mkdir -p $O
timeout -k 10 300 python3 bench/pipe_cmp.py --batch 320 > $O/cmp320.jsonl 2>&1
timeout -k 10 300 python3 bench/pipe_cmp.py --batch 32 > $O/cmp32.jsonl 2>&1
timeout -k 10 300 python3 bench/pipe_cmp.py --batch 32 --dgrad > $O/cmp32d.jsonl 2>&1
