"""Decode-attention sweep (k_attn_decode, the rollout's KV-cache attention + fused out-projection):
KV length t x live rows R at the C3 model (dh 16, H 4, d 256), where the cache read dominates.

    python tools/attn_sweep.py run [--reps 10] [--out gpurun_out/attn_sweep.json]
    python tools/attn_sweep.py summarize gpurun_out/attn_sweep.json <kernel_trace dir> [<pmc FETCH dir> <pmc WRITE dir>]

``run`` builds a C3 learner with Tmax 512, rolls out once (weights packed, caches filled), then for
every (t, R) point makes the first R slots live (alive = 1, the rest dead) and runs the multi-kernel
decode step at position t ``warm + reps`` times; HIP events around every attention launch of the
timed reps (XtrlDecodeDesc.prof_events) give the event time.  Algorithmic bytes per launch as
bench.py's DecodeAttnTimer: per live (row, head) the K and V rows 0..t-1 (2 t dh fp32) + the row's
q|k|v|gate|mix operands + the value-residual row + the K/V append + the output.
``summarize`` assigns the k_attn_decode dispatches of a rocprofv3 --kernel-trace (and optional
--pmc FETCH_SIZE / WRITE_SIZE) run of ``run`` to the points in launch order (the points are run
in a fixed order, (warm + reps) x L dispatches each) and reports the profiler's duration and the
counters' HBM bytes per launch (reads = 2 x FETCH_SIZE, the gfx950 correction of the MI355X guide).
"""
import argparse
import csv
import ctypes as C
import glob
import json
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / 'x-transformers-rl_amd')]

TS = (64, 128, 256, 500)
RS = (256, 1024)
WARM = 2
HBM = 8000.0


def points():
    return [(t, r) for r in RS for t in TS]


def algo_bytes(c, t, R):
    H, dh = c.heads, c.dim_head
    row = 3 * dh + (dh if c.gate_values else 0) + (1 if c.learned_mix else 0)
    vres = dh if c.value_residual else 0
    return 4.0 * R * H * (2 * t * dh + row + vres + 2 * dh + dh)


def run(a):
    import torch
    import bench
    cfg = dict(bench.CONFIGS['c3'], T=512)
    torch.manual_seed(0)
    learner, env = bench.build_learner(cfg, 0, use_graph=False)
    learner.rollout_device(env, 0, 512)      # packs the weights, fills the caches
    torch.cuda.synchronize()
    eng = learner._engine_for(env, 512)
    c = eng.c
    L = c.depth
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * 512 * L)]
    for e in ev:
        e.record()
    torch.cuda.synchronize()
    arr = (C.c_void_p * len(ev))(*[e.cuda_event for e in ev])
    out = []
    for (t, R) in points():
        ms = 0.0
        for rep in range(WARM + a.reps):
            eng.alive.zero_()
            eng.alive[:R] = 1
            eng.lens.fill_(t)
            eng.desc.prof_events = C.cast(arr, C.POINTER(C.c_void_p)) if rep >= WARM else None
            eng.step(t)
            if rep >= WARM:
                torch.cuda.synchronize()
                ms += sum(ev[2 * (t * L + l)].elapsed_time(ev[2 * (t * L + l) + 1]) for l in range(L))
        eng.desc.prof_events = None
        us = ms * 1e3 / (a.reps * L)
        b = algo_bytes(c, t, R)
        out.append(dict(t=t, rows=R, us_event=round(us, 2), bytes=b, gbs_event=round(b / us / 1e3, 1),
                        frac_event=round(b / us / 1e3 / HBM, 4)))
        print(json.dumps(out[-1]), flush=True)
    json.dump(dict(points=out, reps=a.reps, warm=WARM, layers=L), open(a.out, 'w'), indent=1)


def summarize(a):
    meta = json.load(open(a.json))
    L, per = meta['layers'], (meta['warm'] + meta['reps']) * meta['layers']
    skip = meta['warm'] * L

    def dispatches(root, csv_glob, key):
        rows = []
        for f in glob.glob(os.path.join(root, '**', csv_glob), recursive=True):
            for r in csv.DictReader(open(f)):
                if 'k_attn_decode' in r['Kernel_Name']:
                    rows.append(r)
        rows.sort(key=lambda r: int(r[key]))
        return rows

    tr = dispatches(a.trace, '*kernel_trace.csv', 'Start_Timestamp')
    need = per * len(meta['points'])
    # the warm-up rollout's dispatches come first: the sweep's are the last ``need``
    tr = tr[-need:]
    fetch = write = None
    if a.fetch:
        def counter(root, name):
            vals = [r for r in dispatches(root, '*counter_collection.csv', 'Dispatch_Id') if r['Counter_Name'] == name]
            return [float(r['Counter_Value']) * 1024.0 for r in vals][-need:]
        fetch, write = counter(a.fetch, 'FETCH_SIZE'), counter(a.write, 'WRITE_SIZE')
    res = []
    for i, p in enumerate(meta['points']):
        sl = slice(i * per + skip, (i + 1) * per)
        durs = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3 for r in tr[sl]]
        us = sum(durs) / len(durs)
        q = dict(p, us_rocprof=round(us, 2), gbs_rocprof=round(p['bytes'] / us / 1e3, 1),
                 frac_rocprof=round(p['bytes'] / us / 1e3 / HBM, 4))
        if fetch:
            f = sum(fetch[sl]) / len(fetch[sl])
            w = sum(write[sl]) / len(write[sl])
            q.update(hbm_bytes_pmc=round(2 * f + w), gbs_pmc=round((2 * f + w) / us / 1e3, 1),
                     frac_pmc=round((2 * f + w) / us / 1e3 / HBM, 4))
        res.append(q)
        print(json.dumps(q))
    json.dump(dict(meta, points=res), open(a.json.replace('.json', '_summary.json'), 'w'), indent=1)


if __name__ == '__main__':
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest='cmd', required=True)
    r = sub.add_parser('run')
    r.add_argument('--reps', type=int, default=10)
    r.add_argument('--out', default=str(REPO / 'gpurun_out' / 'attn_sweep.json'))
    s = sub.add_parser('summarize')
    s.add_argument('json')
    s.add_argument('trace')
    s.add_argument('fetch', nargs='?')
    s.add_argument('write', nargs='?')
    a = ap.parse_args()
    run(a) if a.cmd == 'run' else summarize(a)
