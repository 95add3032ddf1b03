"""Reader / writer of flax's msgpack state format without flax.

The reference saves env models with ``flax.serialization.to_bytes`` and
loads them with ``from_bytes`` (utils/envmodel.py:38-49,
train_env_model.py:118-123).  flax is not installed here, so this restates
flax.serialization's published format: a msgpack map tree whose array leaves
are ``ExtType(1, packb((shape, dtype_name, raw_bytes)))`` (numpy scalars
ExtType(3, ...)), with arrays above flax's chunk limit split into
``{"__msgpack_chunked_array__": True, "shape": ..., "chunks": {...}}``.
Unpacking executes nothing from the file (plain msgpack decoding).
"""
from __future__ import annotations

import msgpack
import numpy as np

_EXT_NDARRAY, _EXT_COMPLEX, _EXT_NPSCALAR = 1, 2, 3
_CHUNK_KEY = "__msgpack_chunked_array__"


def _ndarray_from_bytes(data: bytes) -> np.ndarray:
    shape, dtype_name, buffer = msgpack.unpackb(data, raw=True)
    if isinstance(dtype_name, bytes):
        dtype_name = dtype_name.decode()
    return np.frombuffer(buffer, dtype=np.dtype(dtype_name)).reshape(tuple(shape)).copy()


def _ext_hook(code, data):
    if code == _EXT_NDARRAY:
        return _ndarray_from_bytes(data)
    if code == _EXT_NPSCALAR:
        return _ndarray_from_bytes(data)[()]
    if code == _EXT_COMPLEX:
        re, im = msgpack.unpackb(data)
        return complex(re, im)
    return msgpack.ExtType(code, data)


def _unchunk(tree):
    if isinstance(tree, dict):
        if tree.get(_CHUNK_KEY):
            chunks = [tree["chunks"][k] for k in sorted(tree["chunks"], key=int)]
            return np.concatenate([c.reshape(-1) for c in chunks]).reshape(tuple(tree["shape"]))
        return {k: _unchunk(v) for k, v in tree.items()}
    return tree


def msgpack_restore(encoded: bytes) -> dict:
    """flax.serialization.msgpack_restore."""
    return _unchunk(msgpack.unpackb(encoded, ext_hook=_ext_hook, raw=False))


def load_flax_msgpack(path) -> dict:
    with open(path, "rb") as f:
        return msgpack_restore(f.read())


def _ext_pack(x):
    if isinstance(x, np.ndarray):
        a = np.ascontiguousarray(x)
        return msgpack.ExtType(_EXT_NDARRAY, msgpack.packb((a.shape, a.dtype.name, a.tobytes()), use_bin_type=True))
    if isinstance(x, np.generic):
        a = np.asarray(x)
        return msgpack.ExtType(_EXT_NPSCALAR, msgpack.packb((a.shape, a.dtype.name, a.tobytes()), use_bin_type=True))
    raise TypeError(f"cannot serialise {type(x)}")


def msgpack_serialize(tree: dict) -> bytes:
    """flax.serialization.msgpack_serialize for numpy trees (no chunking: env
    models are far below flax's chunk size)."""
    return msgpack.packb(tree, default=_ext_pack, strict_types=True)
