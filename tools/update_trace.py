"""Kernel-by-kernel breakdown of one C3 update (run under `rocprofv3 --kernel-trace`).

  python tools/update_trace.py run            # (under rocprofv3) 1 warmup + 1 update, then exit
  python tools/update_trace.py show TRACE.csv # per-phase totals and one minibatch's kernels in order

The measured update is everything from the last rollout-begin / env-reset launches on.
"""
import csv
import sys
from collections import defaultdict
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / 'x-transformers-rl_amd')]


def run(name='c3'):
    import torch
    import bench
    cfg = bench.CONFIGS[name]
    learner, env = bench.build_learner(cfg, 0)
    bench.one_update(learner, env, cfg['T'])
    torch.cuda.synchronize()
    bench.one_update(learner, env, cfg['T'])
    torch.cuda.synchronize()


def short(name):
    name = name.replace('xtrl::(anonymous namespace)::', '').replace('void ', '')
    if name.startswith('k_gemm<'):
        return name.split('(')[0]
    return name.split('(')[0][:60]


def show(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    names = [r['Kernel_Name'] for r in rows]
    dur = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3 for r in rows]
    # the measured update starts at its rollout: the last k_sim_reset / k_rollout_begin pair
    begins = [i for i, n in enumerate(names) if 'k_rollout_begin' in n or 'k_sim_reset' in n]
    start = begins[-1]
    while start - 1 in begins:
        start -= 1
    upd = list(range(start, len(rows)))
    t0 = int(rows[upd[0]]['Start_Timestamp'])
    t1 = int(rows[upd[-1]]['End_Timestamp'])
    print(f'update: {len(upd)} kernels, wall {(t1 - t0) / 1e6:.2f} ms, busy {sum(dur[i] for i in upd) / 1e3:.2f} ms')
    gathers = [i for i in upd if 'k_gather' in names[i] and 'k_gather_rows' not in names[i]]
    # (the reference-mode learn step of the fractal body has no device gather: the learn phase then
    # starts at the GAE launch)
    first = gathers[:1] or [i for i in upd if 'k_hlgauss_gae' in names[i]][:1]
    if first:
        roll = [i for i in upd if i < first[0]]
        learn = [i for i in upd if i >= first[0]]
        for label, seg in (('rollout', roll), ('learn', learn)):
            ts = int(rows[seg[0]]['Start_Timestamp']); te = int(rows[seg[-1]]['End_Timestamp'])
            print(f'{label}: {len(seg)} kernels, wall {(te - ts) / 1e6:.2f} ms, busy {sum(dur[i] for i in seg) / 1e3:.2f} ms')
            agg = defaultdict(lambda: [0, 0.0])
            for i in seg:
                a = agg[short(names[i])]; a[0] += 1; a[1] += dur[i]
            for k, (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:25]:
                print(f'  {us / 1e3:8.2f} ms {n:6d} {us / n:8.1f} us  {k}')
        # GPU idle time in the learn phase (no kernel of any stream running) and where it falls
        seg = learn
        iv = sorted((int(rows[i]['Start_Timestamp']), int(rows[i]['End_Timestamp']), i) for i in seg)
        idle, gaps, cur = 0, [], iv[0][1]
        for s_, e_, i in iv[1:]:
            if s_ > cur:
                idle += s_ - cur
                gaps.append(((s_ - cur) / 1e3, i))
            cur = max(cur, e_)
        gaps.sort(reverse=True)
        print(f'\nlearn idle: {idle / 1e6:.2f} ms in {len(gaps)} gaps; largest:')
        for g_us, i in gaps[:12]:
            print(f'  {g_us:8.1f} us before {short(names[i])}  (after {short(names[i - 1])})')
        # per queue / stream: busy time in the learn phase (the input-gradient chain vs the side stream)
        qkey = 'Stream_Id' if 'Stream_Id' in rows[0] else 'Queue_Id'
        per_q = defaultdict(float)
        for i in seg:
            per_q[rows[i].get(qkey)] += dur[i]
        lw = (int(rows[seg[-1]]['End_Timestamp']) - int(rows[seg[0]]['Start_Timestamp'])) / 1e3
        print(f'learn busy per {qkey} (wall {lw / 1e3:.2f} ms): ' +
              ', '.join(f'{q}: {us / 1e3:.2f} ms' for q, us in sorted(per_q.items(), key=lambda kv: -kv[1])))
        # per stream: the learn kernels by time (the input-gradient chain's stream is the critical path)
        for q in sorted(per_q, key=lambda k: -per_q[k]):
            agg = defaultdict(lambda: [0, 0.0])
            for i in seg:
                if rows[i].get(qkey) == q:
                    a = agg[short(names[i])]; a[0] += 1; a[1] += dur[i]
            print(f'  {qkey} {q}:')
            for k, (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:12]:
                print(f'    {us / 1e3:8.2f} ms {n:6d} {us / n:8.1f} us  {k}')
        # the main stream's kernels by launch shape (kernel, grid): which GEMM shape costs what
        main_q = max(per_q, key=lambda k: per_q[k])
        agg = defaultdict(lambda: [0, 0.0])
        for i in seg:
            if rows[i].get(qkey) == main_q:
                grid = 'x'.join(rows[i].get(f'Grid_Size_{a_}', '?') for a_ in 'XYZ')
                a = agg[(short(names[i]), grid)]; a[0] += 1; a[1] += dur[i]
        print(f'  {qkey} {main_q} by launch shape:')
        for (k, grid), (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:30]:
            print(f'    {us / 1e3:8.2f} ms {n:6d} {us / n:8.1f} us  {k} [{grid}]')
        by_next = defaultdict(float)
        for g_us, i in gaps:
            by_next[short(names[i])] += g_us
        print('idle by the kernel that ends it:')
        for k, v in sorted(by_next.items(), key=lambda kv: -kv[1])[:10]:
            print(f'  {v / 1e3:8.2f} ms  {k}')
        # one minibatch: between the 2nd and 3rd gather
        if len(gathers) > 2:
            a, b = gathers[1], gathers[2]
            ts = int(rows[a]['Start_Timestamp']); te = int(rows[b]['Start_Timestamp'])
            print(f'\nminibatch (gather #2..#3): {b - a} kernels, wall {(te - ts) / 1e3:.1f} us, '
                  f'busy {sum(dur[a:b]):.1f} us')
            qk = 'Stream_Id' if 'Stream_Id' in rows[0] else 'Queue_Id'
            last_end = {}
            idle_q = defaultdict(float)
            for i in range(a, b):
                gap = (int(rows[i]['Start_Timestamp']) - int(rows[i - 1]['End_Timestamp'])) / 1e3
                q = rows[i].get(qk)
                # the gap since this stream's previous kernel ended (its own idle time)
                qgap = (int(rows[i]['Start_Timestamp']) - last_end[q]) / 1e3 if q in last_end else 0.0
                idle_q[q] += max(qgap, 0.0)
                last_end[q] = int(rows[i]['End_Timestamp'])
                grid = 'x'.join(rows[i].get(f'Grid_Size_{a_}', '?') for a_ in 'XYZ')
                print(f'  {dur[i]:8.1f} us  gap {gap:6.1f}  q{q} qgap {qgap:6.1f} at {(int(rows[i]["Start_Timestamp"]) - ts) / 1e3:7.1f}  '
                      f'{short(names[i])} [{grid}]')
            print('  stream idle inside the minibatch: ' + ', '.join(f'{q}: {v:.1f} us' for q, v in idle_q.items()))
        # one decode step: the kernels between two consecutive sampling launches in the rollout
        samples = [i for i in roll if 'k_sample' in names[i] or 'k_heads_sample' in names[i]]
        if len(samples) > 12:
            a, b = samples[10], samples[11]
            ts = int(rows[a]['End_Timestamp']); te = int(rows[b]['End_Timestamp'])
            print(f'\ndecode step (sampling launch #10..#11): {b - a} kernels, wall {(te - ts) / 1e3:.1f} us')
            for i in range(a + 1, b + 1):
                gap = (int(rows[i]['Start_Timestamp']) - int(rows[i - 1]['End_Timestamp'])) / 1e3
                print(f'  {dur[i]:8.1f} us  gap {gap:6.1f}  {short(names[i])}')


if __name__ == '__main__':
    if sys.argv[1] == 'run':
        run(sys.argv[2] if len(sys.argv) > 2 else 'c3')
    else:
        show(sys.argv[2])
