"""Summarise a rocprofv3 --stats kernel_stats.csv per training step."""
import csv
import sys

path = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 7
rows = list(csv.DictReader(open(path)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:int(sys.argv[3]) if len(sys.argv) > 3 else 20]:
    print("%-58s %5d/step %9.1fus avg %7.2fms/step %5.1f%%" % (
        r['Name'][:58], int(r['Calls']) // steps, float(r['AverageNs']) / 1e3,
        float(r['TotalDurationNs']) / 1e6 / steps, 100 * float(r['TotalDurationNs']) / tot))
print('total ms/step %.2f' % (tot / 1e6 / steps))
