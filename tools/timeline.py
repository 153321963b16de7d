"""Print the kernel timeline of bench steps from a rocprofv3 kernel-trace CSV (profiling aid)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
first = sys.argv[2] if len(sys.argv) > 2 else 'k_bd_sha_payload'
idx = [i for i, r in enumerate(rows) if r['Kernel_Name'].startswith(first)]
for s in idx[-3:-1]:
    t0 = int(rows[s]['Start_Timestamp'])
    j = s - 3
    while j < len(rows) and (j <= s or not rows[j]['Kernel_Name'].startswith(first)):
        r = rows[j]
        print("%-26s q%-3s %7.1f %7.1f  dur %6.1f" % (r['Kernel_Name'][:26], r.get('Queue_Id', ''),
              (int(r['Start_Timestamp']) - t0) / 1e3, (int(r['End_Timestamp']) - t0) / 1e3,
              (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3))
        j += 1
    print('---')
