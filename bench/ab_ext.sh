# In-process-box A/B of two builds: bash bench/ab_ext.sh OLD.so TAG
set -e
OLD=$1; O=gpurun_out/ab_$2; mkdir -p $O
for i in 1 2 3; do
 MERCURY_EXT_PATH=$OLD timeout -k 10 120 python3 bench.py --steps 300 --warmup 30 --no-overhead > $O/old$i.json 2>/dev/null
 timeout -k 10 120 python3 bench.py --steps 300 --warmup 30 --no-overhead > $O/new$i.json 2>/dev/null
done
MERCURY_EXT_PATH=$OLD timeout -k 10 300 python3 bench/kernel_sweep.py --batch 320 --kind fwd --pipes 0 > $O/old320.jsonl 2>&1
timeout -k 10 300 python3 bench/kernel_sweep.py --batch 320 --kind fwd --pipes 0 > $O/new320.jsonl 2>&1
MERCURY_EXT_PATH=$OLD timeout -k 10 300 python3 bench/kernel_sweep.py --batch 32 --pipes 0 > $O/old32.jsonl 2>&1
timeout -k 10 300 python3 bench/kernel_sweep.py --batch 32 --pipes 0 > $O/new32.jsonl 2>&1
