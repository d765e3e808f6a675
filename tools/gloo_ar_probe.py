"""2 ranks (gloo, sharing one GPU): time the bucketed gradient all-reduce of the C3 decoder and the C5
fractal body on their real flat layouts, without the learn step around it."""
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'x-transformers-rl_amd'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))


def main():
    dist.init_process_group('gloo')
    rank = dist.get_rank()
    torch.cuda.set_device(0)
    import bench
    from xtrl_amd.distributed import BucketAllReduce
    for cfg in ('c3', 'c5'):
        learner, env = bench.build_learner(bench.CONFIGS[cfg], 0, use_graph=False, world=2)
        agent = learner.agent
        bar = agent.bucket_allreduce()
        buf = agent.flat.grad_ext
        print(f'[{rank}] {cfg}: {buf.numel()} floats, groups {bar.groups if bar else None}', flush=True)
        for e in (bar.events if bar else []):
            e.record()
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(10):
            for e in bar.events:
                e.record()
            bar.run()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 10
        t0 = time.perf_counter()
        for _ in range(10):
            dist.all_reduce(buf)
        torch.cuda.synchronize()
        d1 = (time.perf_counter() - t0) / 10
        print(f'[{rank}] {cfg}: bucketed {1e3 * dt:.1f} ms, one all_reduce {1e3 * d1:.1f} ms per step', flush=True)
        del learner
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
