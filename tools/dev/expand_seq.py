# Per-call expand kernel sequence from a rocprofv3 kernel trace (E<mode>: expand_kernel, R: copy_lane_runs, B: copy_big_runs,
# G: gather_staged, H: handles_to_rows); durations in microseconds.
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
line=[]
for r in rows:
    n=r['Kernel_Name']
    if 'expand_kernel' in n: k='E'+n.split('expand_kernel<')[1][0]
    elif 'copy_lane_runs' in n: k='R'
    elif 'copy_big_runs' in n: k='B'
    elif 'copy_runs' in n: k='R'
    elif 'gather_staged' in n: k='G'
    elif 'handles_to_rows' in n: k='H'
    else: continue
    line.append(f"{k}:{(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3:.0f}")
    if k=='H': print(' '.join(line)); line=[]
