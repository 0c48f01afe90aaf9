"""Per-kernel durations of the last full epoch in a rocprofv3 kernel trace."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
names = [r['Kernel_Name'].replace('frecsys_hip::(anonymous namespace)::', '').split('(')[0]
         .replace('void ', '') for r in rows]
ul = [i for i, n in enumerate(names) if 'loss' in n]
tot = 0.0
for i in range(ul[-2] + 1, ul[-1] + 1):
    r = rows[i]
    ms = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6
    tot += ms
    print('%-28s %8.3f ms  grid %d' % (names[i], ms,
                                        int(r['Grid_Size_X']) // int(r['Workgroup_Size_X'])))
print('sum %.3f ms' % tot)
