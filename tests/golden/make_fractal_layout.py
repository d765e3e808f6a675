"""Writes tests/golden/fractal_easy_layout.json: parameter names / shapes and the fractal config of
the reference's committed checkpoint fractal_experiments/frala_easy_final/final_fractal_agent.pt
(read with torch.load(weights_only=True): no code from the file runs), plus per-tensor sums of the
world-model weights.  Run in the build container, where /root/reference exists:
    python tests/golden/make_fractal_layout.py
"""
import json
from pathlib import Path

import torch

SRC = Path('/root/reference/fractal_experiments/frala_easy_final/final_fractal_agent.pt')
OUT = Path(__file__).resolve().parent / 'fractal_easy_layout.json'

ck = torch.load(SRC, weights_only=True, map_location='cpu')
wm = ck['world_model']
layout = {k: list(v.shape) for k, v in wm.items()}
sums = {k: float(v.double().sum()) for k, v in wm.items()}
json.dump(dict(fractal_config=ck['fractal_config'], agent_config={k: v for k, v in ck['agent_config'].items()},
               layout=layout, sums=sums), OUT.open('w'), indent=1, default=list)
print(OUT, len(layout), 'tensors')
