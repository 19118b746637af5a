import csv, sys, collections
d = sys.argv[1]
rows = list(csv.DictReader(open(d + '/run_kernel_stats.csv')))
tot = sum(float(r['TotalDurationNs']) for r in rows)
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 13
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:30]:
    print(f"{float(r['TotalDurationNs'])/1e6/steps:8.3f}ms/step {float(r['Percentage']):6.2f}% calls={int(r['Calls'])/steps:6.1f}/step avg={float(r['AverageNs'])/1e3:8.1f}us  {r['Name'][:100]}")
print('total ms/step', tot/1e6/steps)
