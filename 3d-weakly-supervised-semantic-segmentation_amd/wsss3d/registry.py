"""Name -> (object, meta) registries with the reference's behaviour
(`utils/registry.py:1-81`): `register(**meta)` as a decorator stores the class
under its __name__ (optionally `name_suffix`), duplicate names are an error,
`get(name)` falls back to `name_3d` and raises KeyError when neither exists.
Encoders carry `embed_length=lambda m: ...` metadata that the task heads read
(`models/MultiLabelContrastive.py:14`)."""
from __future__ import annotations


class Registry:
    def __init__(self, name):
        self._name = name
        self._obj_map = {}

    def _do_register(self, name, obj, suffix=None, **meta):
        if isinstance(suffix, str):
            name = f"{name}_{suffix}"
        if name in self._obj_map:
            raise AssertionError(f"An object named '{name}' was already registered in '{self._name}' registry!")
        self._obj_map[name] = (obj, meta)

    def register(self, obj=None, suffix=None, **meta):
        if obj is not None:
            self._do_register(obj.__name__, obj, suffix)
            return obj

        def deco(o):
            self._do_register(o.__name__, o, suffix, **meta)
            return o

        return deco

    def get(self, name, suffix="3d"):
        hit = self._obj_map.get(name)
        if hit is None:
            hit = self._obj_map.get(f"{name}_{suffix}")
        if hit is None:
            raise KeyError(f"No object named '{name}' found in '{self._name}' registry!")
        return hit

    def __contains__(self, name):
        return name in self._obj_map

    def __iter__(self):
        return iter(self._obj_map.items())

    def keys(self):
        return self._obj_map.keys()


DATASET_REGISTRY = Registry("dataset")
ARCH_REGISTRY = Registry("arch")
MODEL_REGISTRY = Registry("model")
LOSS_REGISTRY = Registry("loss")
METRIC_REGISTRY = Registry("metric")
