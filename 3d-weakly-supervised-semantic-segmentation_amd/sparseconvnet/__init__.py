"""MI355X-native drop-in for the `sparseconvnet` (SCN 0.2) API surface the
reference uses.

`import sparseconvnet as scn` resolves here when
`3d-weakly-supervised-semantic-segmentation_amd/` is on sys.path; every
compute call goes to libmi3dsparse.so (HIP, gfx950) through the C ABI in
include/mi3dsparse.h.
"""
from .sparseConvNetTensor import SparseConvNetTensor
from .metadata import Metadata
from .modules import (AddTable, BatchNormalization, BatchNormLeakyReLU, BatchNormReLU, ConcatTable, Convolution,
                      Deconvolution, Identity, InputLayer, JoinTable, MaxPooling, NetworkInNetwork, OutputLayer,
                      Sequential, SparseToDense, SubmanifoldConvolution, UnPooling, prefetch_metadata)
from .networkArchitectures import FullyConvolutionalNet, FullyConvolutionalNetEncoder, UNet
from .utils import checkpoint_restore, checkpoint_save, is_power2
from . import _lib
from . import weight_images
from . import graphs

# SCN's global work counters (train.py:50-51,86-87): multiply-adds of every
# convolution (rules * nIn * nOut) and output elements of every convolution.
forward_pass_multiplyAdd_count = 0
forward_pass_hidden_states = 0

__all__ = [
    "SparseConvNetTensor", "Metadata", "InputLayer", "OutputLayer", "SubmanifoldConvolution", "Convolution",
    "Deconvolution", "NetworkInNetwork", "UnPooling", "MaxPooling", "BatchNormalization", "BatchNormReLU",
    "BatchNormLeakyReLU", "Sequential", "ConcatTable", "AddTable", "JoinTable", "Identity", "SparseToDense",
    "UNet", "FullyConvolutionalNet", "FullyConvolutionalNetEncoder", "checkpoint_save", "checkpoint_restore",
    "is_power2", "forward_pass_multiplyAdd_count", "forward_pass_hidden_states", "prefetch_metadata",
    "weight_images", "graphs",
]
