"""applestar_amd — MI355X-native AlphaStar-class StarCraft II RL framework.

Capabilities of jaymarichua/Applestar (a DI-star fork), re-designed for AMD Instinct MI355X
(gfx950/CDNA4): PyTorch-ROCm for the module tree, hand-written HIP kernels for the hot ops
(``applestar_amd/csrc``), RCCL over xGMI for the data-parallel learner.
"""
__version__ = '0.1.0'
