# same-box A/B of two extension builds on one preset: bash bench/ab_preset.sh OLD.so CONFIG ROUNDS
set -e
old=$1; cfg=$2; n=${3:-3}; o=gpurun_out/ab_${cfg}; mkdir -p $o
for r in $(seq 1 $n); do
  MERCURY_EXT_PATH=$old timeout -k 10 200 python3 bench.py --config $cfg --steps 100 --warmup 10 --no-overhead > $o/old$r.json 2> $o/old$r.err
  timeout -k 10 200 python3 bench.py --config $cfg --steps 100 --warmup 10 --no-overhead > $o/new$r.json 2> $o/new$r.err
done
python3 - "$o" <<'PY'
import glob, json, sys
o = sys.argv[1]
res = {}
for k in ('old', 'new'):
    res[k] = [json.loads(open(f).read().strip().splitlines()[-1])['ms_per_step']
              for f in sorted(glob.glob('%s/%s*.json' % (o, k)))]
print(json.dumps(res))
json.dump(res, open(o + '/ab.json', 'w'))
PY
