import csv, sys, glob
f = glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1
print('%-9s %6s %8s %6s %s' % ('ms/step', 'calls', 'avg_us', '%', 'kernel'))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    print('%9.3f %6d %8.1f %5.1f%% %s' % (float(r['TotalDurationNs']) / 1e6 / steps, int(r['Calls']),
          float(r['AverageNs']) / 1e3, 100 * float(r['TotalDurationNs']) / tot, r['Name'][:100]))
print('total kernel ms/step', tot / 1e6 / steps)
