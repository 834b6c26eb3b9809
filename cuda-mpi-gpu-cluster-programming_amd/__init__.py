"""anx — an MI355X-native (gfx950) multi-GPU AlexNet-block inference framework.

Same capabilities as the CUDA/MPI course project mykolas-perevicius/CUDA-MPI-GPU-Cluster-Programming
(five staged versions V1..V5 of AlexNet Blocks 1-2 inference), re-designed for MI355X: a C++/HIP
core (``libanx``: MFMA implicit-GEMM convolutions, fused epilogues, an exact row-decomposition
planner, persistent-workspace engines) driven from PyTorch-ROCm, with RCCL over xGMI for the
multi-GPU scatter / halo exchange / gather paths.

Import as ``import anx`` (``anx.py`` at the repository root binds this directory).
"""
from . import config  # noqa: F401
from .config import BLOCK1, BLOCK2, blocks, blocks_dims, flops_per_image  # noqa: F401

__version__ = "0.1.0"


def __getattr__(name):  # lazy heavy imports
    if name == "AlexNetBlocks":
        from .models.alexnet_blocks import AlexNetBlocks
        return AlexNetBlocks
    raise AttributeError(name)
