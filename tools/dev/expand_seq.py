# Per-call expand kernel sequence from a rocprofv3 kernel trace (E<mode>: expand_kernel 0 count / 1 fill /
# 2 stage, R: copy_lane_runs, B: copy_big_runs, G: gather_staged, H: handles_to_rows); durations in
# microseconds, and their sum per call (a call ends with its H).  Usage: expand_seq.py <kernel_trace.csv>
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
line, tot, sums = [], 0.0, []
for r in rows:
    n = r['Kernel_Name']
    if 'expand_kernel' in n:
        k = 'E' + n.split('expand_kernel<')[1][0]
    elif 'copy_lane_runs' in n or 'copy_runs' in n:
        k = 'R'
    elif 'copy_big_runs' in n:
        k = 'B'
    elif 'gather_staged' in n:
        k = 'G'
    elif 'handles_to_rows' in n:
        k = 'H'
    else:
        continue
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    tot += d
    line.append(f"{k}:{d:.0f}")
    if k == 'H':
        print(' '.join(line), f"| sum {tot:.0f}")
        sums.append(tot)
        line, tot = [], 0.0
if sums:
    s = sorted(sums[1:] or sums)
    print(f"calls {len(sums)}, median sum {s[len(s) // 2]:.0f} us (first call excluded)")
