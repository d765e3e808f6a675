"""Idle gaps of the learn stream vs the host (rocprofv3 --kernel-trace --hip-trace):
python tools/gap_host_probe.py <dir>.  Prints, for one minibatch of the last learn, every kernel
with its stream, start (us from the minibatch start), duration, the gap before it on its stream and
when its launch call returned relative to that gap; then, over the whole last learn, the host's lead
(kernel start - its launch call's return: small = the GPU is waiting on the host) and the HIP API
calls that took longer than 40 us (blocking calls: synchronisations, copies, allocations)."""
import csv, glob, sys
from collections import defaultdict
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
# the whole last learn: from the first k_gather of the last learn (32 or more minibatches back)
learn0 = starts[0]
for j in range(len(starts) - 1, 0, -1):   # the last run of gathers not interrupted by a rollout
    seg = kt[starts[j - 1]:starts[j]]
    if any('k_rollout_begin' in r['Kernel_Name'] or 'k_sim_reset' in r['Kernel_Name'] for r in seg):
        learn0 = starts[j]; break
L0, L1 = int(kt[learn0]['Start_Timestamp']), int(kt[-1]['End_Timestamp'])
leads = []
for r in kt[learn0:]:
    a = api.get(r['Correlation_Id'])
    if a:
        leads.append((int(r['Start_Timestamp']) - int(a['End_Timestamp'])) / 1e3)
leads.sort()
if leads:
    q = lambda f: leads[min(len(leads) - 1, int(f * len(leads)))]
    print(f'host lead over the last learn ({len(leads)} kernels): min {leads[0]:.1f} p10 {q(0.1):.1f} '
          f'p50 {q(0.5):.1f} p90 {q(0.9):.1f} us; < 20 us: {sum(1 for x in leads if x < 20)}')
slow = defaultdict(lambda: [0, 0.0])
for r in ht:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    if s >= L0 and e <= L1 and (e - s) > 40e3:
        k = slow[r.get('Function', r.get('Kind', '?'))]; k[0] += 1; k[1] += (e - s) / 1e3
print('HIP API calls > 40 us inside the last learn:')
for name, (n, us) in sorted(slow.items(), key=lambda kv: -kv[1][1]):
    print(f'  {us / 1e3:8.2f} ms  {n:5d}  {name}')
