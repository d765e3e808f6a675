"""torch.profiler view of one C3 learn update (which ATen ops / shapes cost what)."""
import sys
sys.path[:0] = ['.', 'x-transformers-rl_amd']
import torch
from bench import CONFIGS, build_learner, one_update
from torch.profiler import profile, ProfilerActivity

cfg = CONFIGS[sys.argv[1] if len(sys.argv) > 1 else 'c3']
learner, env = build_learner(cfg, 0, use_graph=True)
one_update(learner, env, cfg['T'])
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
    one_update(learner, env, cfg['T'])
    torch.cuda.synchronize()
print(prof.key_averages(group_by_input_shape=True).table(sort_by='cuda_time_total', row_limit=45, max_name_column_width=40,
                                                         max_shapes_column_width=70))
