"""Timeline of the last full epoch in a rocprofv3 kernel trace (overlapped streams):
start/end offsets (us) per kernel and its queue, to find the epoch's critical path."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
names = [r['Kernel_Name'].replace('frecsys_hip::(anonymous namespace)::', '').split('(')[0]
         .replace('void ', '') for r in rows]
ul = [i for i, n in enumerate(names) if 'quad_kernel' in n]
lo, hi = ul[-2] + 1, ul[-1] + 1
t0 = int(rows[lo]['Start_Timestamp'])
for i in range(lo, hi + 1 if hi + 1 < len(rows) else hi):
    r = rows[i]
    s = (int(r['Start_Timestamp']) - t0) / 1e3
    e = (int(r['End_Timestamp']) - t0) / 1e3
    print('q%-3s %-30s %9.1f %9.1f %8.1f us  grid %d' % (
        r.get('Queue_Id', '?'), names[i][:30], s, e, e - s,
        int(r['Grid_Size_X']) // int(r['Workgroup_Size_X'])))
