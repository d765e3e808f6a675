"""Oracle — TEST INFRASTRUCTURE ONLY.

CPU restatement of the reference (tinycrops/x-transformers-rl, snapshot 2025-07-04) Learner hot
path, used as the *checker* for the MI355X product path in ``x-transformers-rl_amd/``.

Who may import this package (and nobody else):
  * ``tests/``                      — parity tests (oracle vs HIP path, oracle vs golden fixtures)
  * ``__graft_entry__.smoke()``     — one tiny decode step checked against the oracle
  * ``bench.py`` ``cpu_baseline``   — the reference CPU Learner restatement, timed beside the GPU

The product (``xtrl_amd``) never imports, links or calls anything here; it fails loudly when its
HIP library is missing instead of falling back to a CPU path.

Modules
  thirdparty.py  restatements of the un-vendored third-party libraries on the path
                 (x-transformers Decoder, hl-gauss-pytorch, assoc-scan, ema-pytorch,
                 adam-atan2-pytorch, einx subset).  Their arithmetic is PARITY UNPINNED — the
                 reference tree holds no vectors for them; every unverifiable choice
                 sits behind a named switch in ``XTConfig`` / ``HLGaussLoss``.
  ref_port.py    restatement of x_transformers_rl.py / evolution.py arithmetic (model glue,
                 distributions, losses, RSNorm, GAE, evolve_, Agent.learn, Learner rollout).
                 PINNED against golden vectors produced by running the reference's own code in
                 this container (tests/golden/make_golden.py; tests/test_oracle_golden.py).
  philox.py      counter-based Philox4x32-10 streams + the synthetic LunarLander-shaped Sim,
                 bit-identical to the HIP implementation (integer arithmetic + exact f32 adds).
  fractal_ref.py fp64-capable restatement of the fractal policy body forward (fractal_rl.py).
"""
