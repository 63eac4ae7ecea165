import glob, json, sys
d = sys.argv[1]
for j in range(1, 20):
    fs = sorted(glob.glob('%s/v%d_*.json' % (d, j)))
    if not fs:
        break
    print(j, [json.loads(open(f).read().strip().splitlines()[-1])['ms_per_step'] for f in fs])
