"""Idle gaps of the learn stream vs the host (rocprofv3 --kernel-trace --hip-trace):
python tools/gap_host_probe.py <dir>.  Prints, for one minibatch of the last learn, every kernel
with its stream, start (us from the minibatch start), duration, the gap before it on its stream and
when its launch call returned relative to that gap."""
import csv, glob, sys
d = sys.argv[1]
kt = list(csv.DictReader(open(glob.glob(f'{d}/**/*kernel_trace.csv', recursive=True)[0])))
ht = list(csv.DictReader(open(glob.glob(f'{d}/**/*hip_api_trace.csv', recursive=True)[0])))
api = {r['Correlation_Id']: r for r in ht}
kt.sort(key=lambda r: int(r['Start_Timestamp']))
short = lambda n: n.replace('void ', '').replace('xtrl::(anonymous namespace)::', '')[:58]
# the minibatch boundaries: k_gather launches (device minibatch assembly)
starts = [i for i, r in enumerate(kt) if 'k_gather' in r['Kernel_Name']]
if len(starts) < 3:
    print('no minibatches found'); sys.exit(0)
i0, i1 = starts[-3], starts[-2]
t0 = int(kt[i0]['Start_Timestamp'])
last_end = {}
for r in kt[:i0]:
    q = r['Stream_Id']; last_end[q] = max(last_end.get(q, 0), int(r['End_Timestamp']))
tot_gap = 0.0
for r in kt[i0:i1]:
    s, e, q = int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Stream_Id']
    prev = last_end.get(q, s)
    gap = (s - prev) / 1e3
    last_end[q] = max(prev, e)
    a = api.get(r['Correlation_Id'])
    launched = (int(a['End_Timestamp']) - prev) / 1e3 if a else float('nan')
    flag = ''
    if gap > 10:
        tot_gap += gap
        flag = 'HOST' if launched > 0 else 'WAIT'
    print(f"{q:>3} {(s - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f} gap {gap:7.1f} call-ret {launched:8.1f} {flag:4s} {short(r['Kernel_Name'])}")
print(f'gaps > 10 us in this minibatch: {tot_gap:.1f} us')
