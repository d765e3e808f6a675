"""xtrl_amd — MI355X-native (gfx950) Learner hot path of x-transformers-rl.

Drop-in names: ``Learner``, ``Agent`` (x_transformers_rl/__init__.py:1-4).  The compute path is
libxtrl_hip.so (HIP kernels for CDNA4, C ABI in include/xtrl_hip.h); PyTorch provides device
memory, streams, autograd for the dense layers and torch.distributed (RCCL) for data parallelism.
"""
from .learner import Agent, Learner, SynthVecSim
from .model import ModelConfig, WorldModelActorCritic

__all__ = ['Learner', 'Agent', 'SynthVecSim', 'ModelConfig', 'WorldModelActorCritic']
