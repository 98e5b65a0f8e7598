"""Per-launch durations (us) of one kernel in the last kernel trace under gpurun_out/kt (tools/prof_fused.sh)."""
import csv,sys,glob
f=glob.glob('gpurun_out/kt/**/*kernel_trace.csv',recursive=True)[0]
rows=[r for r in csv.DictReader(open(f)) if sys.argv[1] in r['Kernel_Name']]
d=[(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3 for r in rows][-16:]
print(sys.argv[1], [round(x,1) for x in d])
