"""Host-side mirror of the reference's model layer for the encoder hot path:
registry (`utils/registry.py`), encoder plugin surface
(`models/SparseConvNet.py`), task heads and losses
(`models/MultiLabelContrastive.py`, `utils/loss.py`), the synthetic batch
producer (`dataset/data.py` transforms), the fixed-shape caption tokenizer
(`dataset/dataset_utils/text_transform_builder.py`) and the data-parallel driver and the device-side validation accumulation
(`train.py:94-116`)."""
from .edict import EasyDict
from .registry import LOSS_REGISTRY, MODEL_REGISTRY, Registry
from . import encoders, evaluate, heads, text, tokenizer  # noqa: F401  (registers the classes)
from .encoders import SparseConvBase_, segment_mean
from .tokenizer import text_transform

__all__ = ["EasyDict", "Registry", "MODEL_REGISTRY", "LOSS_REGISTRY", "SparseConvBase_", "segment_mean",
           "text_transform"]
