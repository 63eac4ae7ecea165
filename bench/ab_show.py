import glob, json, sys
d = sys.argv[1]
for k in ('old', 'new'):
    v = [json.loads(open(f).read().strip().splitlines()[-1])['ms_per_step'] for f in sorted(glob.glob('%s/%s[0-9].json' % (d, k)))]
    print(k, v)
for f in sorted(glob.glob(d + '/*.jsonl')):
    print(f, open(f).read().strip().splitlines()[-1])
